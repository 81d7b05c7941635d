#!/usr/bin/env python3
"""Diagnostic (GPU box): the discriminator plan alone vs fp64 autograd of the oracle's
NLayerDiscriminator, plus run-to-run determinism of the whole step."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mra-gan_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from golden_util import inputs, load  # noqa: E402
from oracle import cyclegan_oracle as O  # noqa: E402
from test_step_gpu import build_model  # noqa: E402


def rel(a, b):
    return float((a.double().cpu() - b.double().cpu()).norm() / max(float(b.double().norm()), 1e-300))


def d_only(model, S, b):
    from mragan_hip import ops
    net = model.netD_A
    plan = net.plan
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2 * b, 1, S, S, S, generator=g)
    xg = x.permute(0, 2, 3, 4, 1).contiguous().cuda()
    from models.networks3D import ensure_flat
    ensure_flat(net)
    net._flat_grad.zero_()
    ctx = plan.forward(xg)
    dl = torch.empty_like(ctx.out)
    slot = torch.zeros(1, device="cuda")
    ops.gan_loss(ctx.out[:b], 1.0, False, 0.5, slot, dl[:b])
    ops.gan_loss(ctx.out[b:], 0.0, False, 0.5, slot, dl[b:], loss_accumulate=True)
    plan.backward(ctx, [dl], need_wgrad=True, need_input_grad=False)
    torch.cuda.synchronize()
    # fp64 reference
    layers = O.nlayer_discriminator_layers(1, model.opt.ndf, 3, True)
    state = {k: v.detach().cpu().double().clone() for k, v in net.state_dict().items()}
    params = {k: state[k].clone().requires_grad_() for k in state if k.endswith("weight") or k.endswith("bias")}
    xd = x.double()
    pr = O.discriminator_forward(state, params, layers, xd[:b])
    pf = O.discriminator_forward(state, params, layers, xd[b:])
    loss = 0.5 * (O.gan_loss(pr, True, False) + O.gan_loss(pf, False, False))
    loss.backward()
    print("D loss ours", float(slot), "ref", float(loss))
    for k, p in net.named_parameters():
        print(f"  {k:20s} {rel(p.grad, params[k].grad):.2e}")


def d_phase_sensitivity(meta):
    """fp64 D-phase gradients evaluated on (a) the fp64 oracle's fake volume and (b) ours."""
    from golden_util import CASE_KW
    m = build_model(meta, "/tmp/diag_ck_s")
    init = {n: {k: v.detach().cpu().double().clone() for k, v in getattr(m, "net" + n).state_dict().items()}
            for n in ("D_A", "D_B")}
    A, B = inputs(meta, 0)
    m.set_input([A, B])
    m.optimize_parameters()
    torch.cuda.synchronize()
    torch.manual_seed(meta["seed"])
    orc = O.CycleGANOracle(dtype=torch.float64, pool_rng=random.Random(meta["seed"]), **CASE_KW[meta_name])
    orc.optimize_parameters(A, B)
    layers = O.nlayer_discriminator_layers(meta["nc"], m.opt.ndf, 3, True)
    for dn, real, fake_ours, fake_orc in (("D_A", B, m.fake_B, orc.fake_B), ("D_B", A, m.fake_A, orc.fake_A)):
        res = {}
        for tag, fake in (("orc", fake_orc), ("ours", fake_ours.detach().double().cpu())):
            state = {k: v.clone() for k, v in init[dn].items()}
            params = {k: state[k].clone().requires_grad_() for k in state if k.endswith("weight") or k.endswith("bias")}
            loss = 0.5 * (O.gan_loss(O.discriminator_forward(state, params, layers, real.double()), True, False) +
                          O.gan_loss(O.discriminator_forward(state, params, layers, fake), False, False))
            loss.backward()
            res[tag] = {k: p.grad for k, p in params.items()}
        net = getattr(m, "net" + dn)
        for k, p in net.named_parameters():
            if not k.endswith("weight"):
                continue
            print(f"{dn} {k:16s} ours-vs-fp64(our fakes) {rel(p.grad, res['ours'][k]):.2e}   "
                  f"fp64(our fakes)-vs-fp64(oracle fakes) {rel(res['ours'][k], res['orc'][k]):.2e}")
        # how many first-layer pre-activations sit near zero
        y = O.F.conv3d(fake_orc, init[dn]["model.0.weight"], init[dn]["model.0.bias"], stride=2, padding=1)
        print(dn, "first-layer |pre-activation| < 1e-5:", int((y.abs() < 1e-5).sum()), "of", y.numel())


meta_name = None


def main():
    global meta_name
    name = sys.argv[1] if len(sys.argv) > 1 else "step_r9_s32_b1"
    meta_name = name
    z, meta = load(name)
    model = build_model(meta, "/tmp/diag_ck")
    d_only(model, meta["S"], meta["B"])
    d_phase_sensitivity(meta)
    # determinism: two identical models, one step each
    grads = []
    for rep in range(2):
        m = build_model(meta, f"/tmp/diag_ck{rep}")
        A, B = inputs(meta, 0)
        m.set_input([A, B])
        m.optimize_parameters()
        torch.cuda.synchronize()
        grads.append({n: getattr(m, "net" + n)._flat_grad.clone() for n in ("G_A", "G_B", "D_A", "D_B")})
    for n in grads[0]:
        d = (grads[0][n] - grads[1][n]).abs().max().item()
        print("determinism", n, "max |diff| =", d)


if __name__ == "__main__":
    main()
