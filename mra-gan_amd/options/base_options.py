"""Command-line options — drop-in for the reference's options/base_options.py.

Flag names, types and defaults are those of the reference (options/base_options.py:12-57),
including its quirks (netG default resnet_6blocks, ngf = ndf = 32, --patch_size without a
type, gpu_ids forced to 0 by parse()).  Two-pass parsing lets the selected model add its own
flags (`modify_commandline_options`), and parse() writes `<checkpoints_dir>/<name>/opt.txt`.
"""
import argparse
import os

import torch

import models
from utils.utils import mkdirs

# (flag, add_argument kwargs) — order and defaults as in the reference
BASE_FLAGS = [
    ('--data_path', dict(type=str, default='/media/chayanin/Storage/chin/data2021/syn2agi_GAN/train_half/',
                         help='Train images path')),
    ('--val_path', dict(type=str, default='/media/chayanin/Storage/chin/data2021/syn2agi_GAN/test_half/',
                        help='Validation images path')),
    ('--batch_size', dict(type=int, default=1, help='input batch size')),
    ('--patch_size', dict(default=[128 / 2, 128 / 2, 64 / 1], help='Size of the patches extracted from the image')),
    ('--input_nc', dict(type=int, default=1, help='# of input image channels')),
    ('--output_nc', dict(type=int, default=1, help='# of output image channels')),
    ('--resample', dict(default=False, help='Decide or not to rescale the images to a new resolution')),
    ('--new_resolution', dict(default=(1, 1, 1), help='New resolution (if you want to resample the data again)')),
    ('--min_pixel', dict(default=0.1, help='Percentage of minimum non-zero pixels in the cropped label')),
    ('--drop_ratio', dict(default=0, help='Probability to drop a cropped area if the label is empty')),
    ('--ngf', dict(type=int, default=32, help='# of gen filters in first conv layer')),
    ('--ndf', dict(type=int, default=32, help='# of discrim filters in first conv layer')),
    ('--netD', dict(type=str, default='n_layers', help='selects model to use for netD')),
    ('--n_layers_D', dict(type=int, default=3, help='only used if netD==n_layers')),
    ('--netG', dict(type=str, default='resnet_6blocks', help='selects model to use for netG')),
    ('--gpu_ids', dict(default='0', help='gpu ids: e.g. 0  0,1,2, 0,2. use -1 for CPU')),
    ('--name', dict(type=str, default='experiment_name', help='name of the experiment (checkpoint sub-directory)')),
    ('--model', dict(type=str, default='cycle_gan', help='chooses which model to use. cycle_gan')),
    ('--which_direction', dict(type=str, default='AtoB', help='AtoB or BtoA (keep it AtoB)')),
    ('--checkpoints_dir', dict(type=str, default='./checkpoints', help='models are saved here')),
    ('--workers', dict(default=0, type=int, help='number of data loading workers')),
    ('--norm', dict(type=str, default='instance', help='instance normalization or batch normalization')),
    ('--no_dropout', dict(action='store_true', help='no dropout for the generator')),
    ('--init_type', dict(type=str, default='normal', help='network initialization [normal|xavier|kaiming|orthogonal]')),
    ('--init_gain', dict(type=float, default=0.02, help='scaling factor for normal, xavier and orthogonal.')),
    ('--verbose', dict(action='store_true', help='if specified, print more debugging information')),
    ('--suffix', dict(default='', type=str, help='customized suffix: opt.name = opt.name + suffix')),
    # engine-only flag (not in the reference): contraction precision of the dense MFMA convolutions
    ('--conv_precision', dict(type=str, default='f32', choices=['f32', 'bf16x3', 'bf16', 'fp16'],
                              help='f32: exact fp32 MFMA; bf16x3: split-bf16 MFMA (fp32-grade); bf16 / fp16: one '
                                   'MFMA per product on rounded operands; all with fp32 accumulation, fp32 '
                                   'tensors and fp32 master weights / Adam')),
    # engine-only flag: static loss scale of the fp16 mode (gradients stay in fp16's normal range)
    ('--loss_scale', dict(type=float, default=1024.0,
                          help='fp16 conv precision: gradients are computed scaled by this factor and '
                               'unscaled inside the optimizer (ignored in the other precisions)')),
    # engine-only flag: run optimize_parameters() as captured HIP graphs after its first step
    ('--no_cuda_graph', dict(action='store_true',
                             help='launch every kernel of the training step from Python instead of replaying '
                                  'the step captured as HIP graphs')),
    # engine-only flag: the G_A / G_B (and D_A / D_B) chains of a step are independent until their
    # weight gradients meet; by default they run on two HIP streams (two branches of the graph)
    ('--single_stream', dict(action='store_true',
                             help='issue the whole training step on one HIP stream (no G_A / G_B, D_A / D_B '
                                  'overlap)')),
]


class BaseOptions():
    def __init__(self):
        self.initialized = False

    def initialize(self, parser):
        for flag, kw in BASE_FLAGS:
            parser.add_argument(flag, **kw)
        self.initialized = True
        return parser

    def gather_options(self):
        if not self.initialized:
            parser = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
            parser = self.initialize(parser)
        opt, _ = parser.parse_known_args()
        # second pass: the selected model's own flags / defaults
        parser = models.get_option_setter(opt.model)(parser, self.isTrain)
        opt, _ = parser.parse_known_args()
        self.parser = parser
        return parser.parse_args()

    def print_options(self, opt):
        lines = ['----------------- Options ---------------']
        for k, v in sorted(vars(opt).items()):
            default = self.parser.get_default(k)
            comment = '\t[default: %s]' % str(default) if v != default else ''
            lines.append('{:>25}: {:<30}{}'.format(str(k), str(v), comment))
        lines.append('----------------- End -------------------')
        message = '\n'.join(lines)
        print(message)
        expr_dir = os.path.join(opt.checkpoints_dir, opt.name)
        mkdirs(expr_dir)
        with open(os.path.join(expr_dir, 'opt.txt'), 'wt') as f:
            f.write(message)
            f.write('\n')

    def parse(self):
        opt = self.gather_options()
        opt.isTrain = self.isTrain
        if opt.suffix:
            opt.name = opt.name + ('_' + opt.suffix.format(**vars(opt)))
        self.print_options(opt)
        # the reference forces GPU 0 (base_options.py:122-123); with one process per GPU the
        # local rank selects the device
        opt.gpu_ids = 0
        if torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        self.opt = opt
        return self.opt
