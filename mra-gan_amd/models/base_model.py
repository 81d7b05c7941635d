"""BaseModel lifecycle — drop-in for the reference's models/base_model.py (lines 7-171).

Same method names and behaviour: setup (schedulers, optional load), eval/test, visuals and
loss getters, checkpoint save/load with the reference's file naming
('%s_net_%s.pth' % (epoch, name)) and state_dict keys, set_requires_grad.
"""
import os
from collections import OrderedDict

import torch

from models import networks3D

device = networks3D.device


class BaseModel:

    @staticmethod
    def modify_commandline_options(parser, is_train):
        return parser

    def name(self):
        return 'BaseModel'

    def initialize(self, opt):
        self.opt = opt
        self.gpu_ids = opt.gpu_ids
        self.isTrain = opt.isTrain
        # inputs and nets live on the HIP device whenever one is present
        self.device = device
        self.save_dir = os.path.join(opt.checkpoints_dir, opt.name)
        self.loss_names = []
        self.model_names = []
        self.visual_names = []
        self.image_paths = []

    def set_input(self, input):
        self.input = input

    def forward(self):
        pass

    def setup(self, opt, parser=None):
        if self.isTrain:
            self.schedulers = [networks3D.get_scheduler(optimizer, opt) for optimizer in self.optimizers]
        if not self.isTrain or opt.continue_train:
            self.load_networks(opt.which_epoch)
        self.print_networks(opt.verbose)

    def eval(self):
        for name in self.model_names:
            if isinstance(name, str):
                getattr(self, 'net' + name).eval()

    def test(self):
        with torch.no_grad():
            self.forward()

    def get_image_paths(self):
        return self.image_paths

    def optimize_parameters(self):
        pass

    def update_learning_rate(self):
        for scheduler in self.schedulers:
            scheduler.step()
        lr = self.optimizers[0].param_groups[0]['lr']
        print('learning rate = %.7f' % lr)

    def get_current_visuals(self):
        out = OrderedDict()
        for name in self.visual_names:
            if isinstance(name, str):
                out[name] = getattr(self, name)
        return out

    def get_current_losses(self):
        out = OrderedDict()
        for name in self.loss_names:
            if isinstance(name, str):
                out[name] = float(getattr(self, 'loss_' + name))
        return out

    def sync_running_stats(self):
        """Data-parallel runs: every rank updates the InstanceNorm running statistics from its
        own patches only (weights stay identical through the gradient all-reduce).  Average them
        over the ranks — the statistics of the global batch's calls — so every rank holds, and
        saves, the same buffers.  No-op on a single process."""
        try:
            import torch.distributed as dist
        except ImportError:
            return
        if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return
        world = dist.get_world_size()
        for name in self.model_names:
            if isinstance(name, str):
                for k, buf in getattr(self, 'net' + name).named_buffers():
                    if k.endswith('running_mean') or k.endswith('running_var'):
                        dist.all_reduce(buf)
                        buf.div_(world)

    def save_networks(self, which_epoch):
        """Writes '<epoch>_net_<name>.pth' = the net's state_dict on CPU (reference :89-112).
        The net itself is not moved (its parameters live in flat device buffers).  Data parallel:
        average the running statistics with sync_running_stats() on EVERY rank first (a
        collective), then save from one rank (train.py does both)."""
        os.makedirs(self.save_dir, exist_ok=True)
        for name in self.model_names:
            if isinstance(name, str):
                net = getattr(self, 'net' + name)
                sd = net.state_dict()
                for k in list(sd.keys()):
                    sd[k] = sd[k].detach().cpu().clone()
                torch.save(sd, os.path.join(self.save_dir, '%s_net_%s.pth' % (which_epoch, name)))

    def _patch_instance_norm_state_dict(self, state_dict, module, keys, i=0):
        """Drop InstanceNorm entries the module does not track (reference :114-127)."""
        key = keys[i]
        if i + 1 == len(keys):
            if module.__class__.__name__.startswith('InstanceNorm'):
                if key in ('running_mean', 'running_var') and getattr(module, key) is None:
                    state_dict.pop('.'.join(keys))
                if key == 'num_batches_tracked':
                    state_dict.pop('.'.join(keys))
        else:
            self._patch_instance_norm_state_dict(state_dict, getattr(module, key), keys, i + 1)

    def load_networks(self, which_epoch):
        for name in self.model_names:
            if isinstance(name, str):
                path = os.path.join(self.save_dir, '%s_net_%s.pth' % (which_epoch, name))
                net = getattr(self, 'net' + name)
                print('loading the model from %s' % path)
                state_dict = torch.load(path, map_location=str(self.device), weights_only=True)
                if hasattr(state_dict, '_metadata'):
                    del state_dict._metadata
                for key in list(state_dict.keys()):
                    self._patch_instance_norm_state_dict(state_dict, net, key.split('.'))
                net.load_state_dict(state_dict)

    def print_networks(self, verbose):
        print('---------- Networks initialized -------------')
        for name in self.model_names:
            if isinstance(name, str):
                net = getattr(self, 'net' + name)
                num_params = sum(p.numel() for p in net.parameters())
                if verbose:
                    print(net)
                print('[Network %s] Total number of parameters : %.3f M' % (name, num_params / 1e6))
        print('-----------------------------------------------')

    def set_requires_grad(self, nets, requires_grad=False):
        if not isinstance(nets, list):
            nets = [nets]
        for net in nets:
            if net is not None:
                for param in net.parameters():
                    param.requires_grad = requires_grad
