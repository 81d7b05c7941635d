"""Drop-in for the reference's train.py: the epoch / iteration loop of train.py:78-147 with the
MONAI loader replaced by the device patch sampler (mragan_hip/patch_sampler.py; train.py:35-52).

    python train.py --data_path <dir with images/ and labels/> --netG resnet_9blocks --name <exp> \
                    [--patch_size ...] [--conv_precision bf16x3] ...

Same options (TrainOptions), same loss_log.txt / stdout lines (utils/visualizer.py), same
checkpoint cadence ('latest' every save_latest_freq iterations, '<epoch>' + 'latest' every
save_epoch_freq epochs) and LambdaLR update per epoch.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from models import create_model  # noqa: E402
from options.train_options import TrainOptions  # noqa: E402
from utils.visualizer import Visualizer  # noqa: E402


def _rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def save(model, *tags):
    """Checkpoint: every rank averages the InstanceNorm running statistics (a collective, so all
    ranks call this at the same iteration), rank 0 writes the files."""
    model.sync_running_stats()
    if _rank() == 0:
        for t in tags:
            model.save_networks(t)


def train(opt, sampler, model=None, log=print):
    """train.py:70-147 over `sampler` (yields dict(image=..., label=...) batches)."""
    if model is None:
        model = create_model(opt)
        model.setup(opt)
        if opt.epoch_count > 1:
            model.load_networks(opt.epoch_count)
    visualizer = Visualizer(opt)
    total_steps = 0
    for epoch in range(opt.epoch_count, opt.niter + opt.niter_decay + 1):
        epoch_start_time = time.time()
        iter_data_time = time.time()
        epoch_iter = 0
        for i, patch_s in enumerate(sampler):
            iter_start_time = time.time()
            if total_steps % opt.print_freq == 0:
                t_data = iter_start_time - iter_data_time
            visualizer.reset()
            total_steps += opt.batch_size
            epoch_iter += opt.batch_size
            model.set_input([patch_s['image'], patch_s['label']])
            model.optimize_parameters()
            if total_steps % opt.print_freq == 0:
                losses = model.get_current_losses()
                t = (time.time() - iter_start_time) / opt.batch_size
                visualizer.print_current_losses(epoch, epoch_iter, losses, t, t_data)
            if total_steps % opt.save_latest_freq == 0:
                log('saving the latest model (epoch %d, total_steps %d)' % (epoch, total_steps))
                save(model, 'latest')
            iter_data_time = time.time()
        if epoch % opt.save_epoch_freq == 0:
            log('saving the model at the end of epoch %d, iters %d' % (epoch, total_steps))
            save(model, 'latest', epoch)
        log('End of epoch %d / %d \t Time Taken: %d sec' %
            (epoch, opt.niter + opt.niter_decay, time.time() - epoch_start_time))
        model.update_learning_rate()
    return model


if __name__ == '__main__':
    import torch
    from mragan_hip.patch_sampler import GpuPatchSampler
    opt = TrainOptions().parse()
    patch = [int(p) for p in opt.patch_size]
    sampler = GpuPatchSampler.from_folder(opt.data_path, patch, torch.device("cuda"), batch_size=opt.batch_size,
                                          num_samples=2)
    train(opt, sampler)
