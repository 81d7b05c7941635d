"""Test options — drop-in for the reference's options/test_options.py (lines 5-20)."""
from options.base_options import BaseOptions

TEST_FLAGS = [
    ("--image", dict(type=str, default='/media/chayanin/Storage/chin/data2021/syn2agi_GAN/test/labels/fake_MRA_use_GB_340.nii')),
    ("--result", dict(type=str,
                      default='/media/chayanin/Storage/chin/data2021/syn2agi_GAN/test/labels/recon_Bi_use_GA_340.nii',
                      help='path to the .nii result to save')),
    ('--phase', dict(type=str, default='test', help='test')),
    ('--which_epoch', dict(type=str, default='latest', help='which epoch to load? set to latest to use latest cached model')),
    ("--stride_inplane", dict(type=int, nargs=1, default=32, help="Stride size in 2D plane")),
    ("--stride_layer", dict(type=int, nargs=1, default=32, help="Stride size in z direction")),
]


class TestOptions(BaseOptions):
    def initialize(self, parser):
        parser = BaseOptions.initialize(self, parser)
        for flag, kw in TEST_FLAGS:
            parser.add_argument(flag, **kw)
        parser.set_defaults(model='test')
        self.isTrain = False
        return parser
