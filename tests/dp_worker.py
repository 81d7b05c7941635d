"""One rank of the 2-rank data-parallel rehearsal of CycleGANModel.optimize_parameters()
(tests/test_dp_gpu.py): run under `python -m torch.distributed.run --nproc-per-node 2`, gloo
process group, every rank on cuda:0 (one MI355X box), each rank stepping ITS patch of a 2-patch
batch through the model's real data-parallel branch (G all-reduce overlapped with the D phase,
both Adam steps after it; eager first step, HIP-graph replays after unless --no_cuda_graph).
Rank 0 writes losses (mean over ranks), parameters and running statistics (averaged over ranks
by sync_running_stats) to --out."""
import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mra-gan_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MODEL_ARGV = ["--netG", "resnet_6blocks", "--ngf", "8", "--ndf", "8", "--batch_size", "1"]
SEED, S, STEPS = 21, 24, 4


def build(ckdir, extra, batch):
    from models import create_model
    from options.train_options import TrainOptions
    argv = sys.argv
    try:
        sys.argv = ["train.py", "--checkpoints_dir", ckdir] + MODEL_ARGV + list(extra)
        opt = TrainOptions().gather_options()
    finally:
        sys.argv = argv
    opt.isTrain, opt.gpu_ids = True, 0
    torch.manual_seed(SEED)
    random.seed(SEED)
    return create_model(opt)


def batch_inputs(step):
    from oracle.cyclegan_oracle import synthetic_pair
    return synthetic_pair((2, 1, S, S, S), 500 + step)


def snapshot(model):
    out = {}
    for n in ("G_A", "G_B", "D_A", "D_B"):
        for k, v in getattr(model, "net" + n).state_dict().items():
            out[f"{n}/{k}"] = v.detach().cpu().clone()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--extra", default="")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    model = build(f"/tmp/mragan_dp_{rank}", a.extra.split(), 1)
    model.setup(model.opt)
    losses = []
    state1 = None
    for step in range(STEPS):
        A, B = batch_inputs(step)
        model.set_input([A[rank:rank + 1], B[rank:rank + 1]])
        model.optimize_parameters()
        mine = torch.tensor(list(model.get_current_losses().values()), dtype=torch.float64)
        dist.all_reduce(mine)
        losses.append(mine / world)
        if step == 0:
            model.sync_running_stats()     # averaging is linear: doing it now changes nothing later
            state1 = snapshot(model)
    assert model._dist, "the data-parallel branch did not engage"
    model.sync_running_stats()
    torch.cuda.synchronize()
    if rank == 0:
        torch.save(dict(losses=torch.stack(losses), state=snapshot(model), state1=state1,
                        graphed=model._graphs is not None), a.out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
