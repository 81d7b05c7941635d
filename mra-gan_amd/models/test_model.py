"""TestModel — drop-in for the reference's models/test_model.py (lines 7-48): one generator
(`--model test`, loaded from '<which_epoch>_net_G<model_suffix>.pth'), forward only.

`forward()` runs the generator on `real_A` through the HIP engine exactly as the reference's
does through torch (train-mode InstanceNorm: the reference never calls eval() in test.py, so the
per-patch statistics are used and the running buffers are updated).  Whole-volume sliding-window
inference on the device is `mragan_hip.sliding_window.inference_volume(model, ...)` (test.py)."""
from models import networks3D
from models.base_model import BaseModel
from models.cycle_gan_model import CycleGANModel

device = networks3D.device


class TestModel(BaseModel):
    def name(self):
        return 'TestModel'

    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        assert not is_train, 'TestModel cannot be used in train mode'
        parser = CycleGANModel.modify_commandline_options(parser, is_train=False)
        parser.set_defaults(dataset_mode='single')
        parser.add_argument('--model_suffix', type=str, default='',
                            help='In checkpoints_dir, [which_epoch]_net_G[model_suffix].pth will'
                            ' be loaded as the generator of TestModel')
        return parser

    def initialize(self, opt):
        assert (not opt.isTrain)
        BaseModel.initialize(self, opt)
        from mragan_hip import ops
        ops.set_conv_precision(getattr(opt, 'conv_precision', 'f32'))
        self.loss_names = []
        self.visual_names = ['real_A', 'fake_B']
        self.model_names = ['G' + opt.model_suffix]
        self.netG = networks3D.define_G(opt.input_nc, opt.output_nc, opt.ngf, opt.netG,
                                        opt.norm, not opt.no_dropout, opt.init_type, opt.init_gain, self.gpu_ids)
        # assigns the model to self.netG_[suffix] so that BaseModel.load_networks finds it
        setattr(self, 'netG' + opt.model_suffix, self.netG)

    def set_input(self, input):
        self.real_A = input.to(self.device)

    def forward(self):
        self.fake_B = self.netG(self.real_A.to(device))
