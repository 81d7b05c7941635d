"""Training options — drop-in for the reference's options/train_options.py (lines 5-26).
Note the reference quirk kept here: --no_lsgan is `store_false`, so the default trains a
vanilla (BCE + sigmoid) GAN and passing --no_lsgan switches to LSGAN."""
from options.base_options import BaseOptions

TRAIN_FLAGS = [
    ('--print_freq', dict(type=int, default=100, help='frequency of showing training results on console')),
    ('--save_latest_freq', dict(type=int, default=1000, help='frequency of saving the latest results')),
    ('--save_epoch_freq', dict(type=int, default=200, help='frequency of saving checkpoints at the end of epochs')),
    ('--continue_train', dict(action='store_true', help='continue training: load the latest model')),
    ('--epoch_count', dict(type=int, default=1, help='the starting epoch count')),
    ('--phase', dict(type=str, default='train', help='train, val, test, etc')),
    ('--which_epoch', dict(type=str, default='latest', help='which epoch to load? set to latest to use latest cached model')),
    ('--niter', dict(type=int, default=500, help='# of iter at starting learning rate')),
    ('--niter_decay', dict(type=int, default=100, help='# of iter to linearly decay learning rate to zero')),
    ('--beta1', dict(type=float, default=0.5, help='momentum term of adam')),
    ('--lr', dict(type=float, default=0.0002, help='initial learning rate for adam')),
    ('--no_lsgan', dict(action='store_false', help='do *not* use least square GAN, if false, use vanilla GAN')),
    ('--pool_size', dict(type=int, default=50, help='the size of image buffer that stores previously generated images')),
    ('--no_html', dict(action='store_true', help='do not save intermediate training results')),
    ('--lr_policy', dict(type=str, default='lambda', help='learning rate policy: lambda|step|plateau|cosine')),
    ('--lr_decay_iters', dict(type=int, default=50, help='multiply by a gamma every lr_decay_iters iterations')),
]


class TrainOptions(BaseOptions):
    def initialize(self, parser):
        parser = BaseOptions.initialize(self, parser)
        for flag, kw in TRAIN_FLAGS:
            parser.add_argument(flag, **kw)
        self.isTrain = True
        return parser
