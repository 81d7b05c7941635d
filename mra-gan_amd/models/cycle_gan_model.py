"""CycleGANModel — drop-in for the reference's models/cycle_gan_model.py (lines 38-240).

Same options, attributes (netG_A/netG_B/netD_A/netD_B, real_A/fake_B/rec_A/idt_A/...,
loss_* , optimizers) and method names.  `optimize_parameters()` computes the same step —
6 generator and 6 discriminator forward/backward passes, both Adam updates, the image pools
and the InstanceNorm running statistics — but as a fused schedule on the HIP engine:

  G passes batched where the reference makes independent calls (InstanceNorm is per
  instance, so this is exact):   G_A([real_A; real_B]) → [fake_B; idt_A]
                                 G_B([real_B; real_A]) → [fake_A; idt_B]
                                 G_B(fake_B) → rec_A,  G_A(fake_A) → rec_B
  D passes batched:              D_A([real_B; pool(fake_B)]), D_B([real_A; pool(fake_A)])
  running stats:                 applied afterwards in the reference's call order.

Multi-GPU (one process per GPU, torch.distributed over RCCL): each rank takes its own patch
batch; the G gradient all-reduce is launched right after backward_G and overlaps the whole D
phase (which only needs pre-update G outputs and D weights), then both optimizers step.
Reordering "G step, then D phase" → "D phase, then G step" is exact for the same reason.
"""
import itertools
import random
from collections import OrderedDict

import torch

from . import networks3D
from .base_model import BaseModel

device = networks3D.device
# A/B switch: MRAGAN_NO_GRAPH_CACHE=1 keeps only the latest capture (round-2 behaviour)
_NO_GRAPH_CACHE = bool(int(__import__("os").environ.get("MRAGAN_NO_GRAPH_CACHE", "0") or "0"))
# A/B switch: MRAGAN_TWO_PHASE=1 runs the D phase after the whole G phase (rounds 1-5) instead of
# beside the G backward on two more streams (single GPU, two lanes)
_TWO_PHASE = __import__("os").environ.get("MRAGAN_TWO_PHASE") is not None
# A/B switch: MRAGAN_FROZEN_D_ON_LANES=1 keeps the frozen discriminator passes of backward_G on the
# lanes, ahead of the cycle-pass backwards (the overlapped schedule then moves only the D phase)
_FROZEN_D_ON_LANES = __import__("os").environ.get("MRAGAN_FROZEN_D_ON_LANES") is not None
# A/B switch: MRAGAN_ADAM_AFTER=1 runs the four Adam updates after the step's graph (rounds 1-5)
_ADAM_AFTER = __import__("os").environ.get("MRAGAN_ADAM_AFTER") is not None
# A/B switch: MRAGAN_PACK_AT_START=1 repacks the generators' weights at the start of each lane (rounds
# 1-6 first session) instead of right after their Adam update at the end of the previous step
_PACK_AT_START = __import__("os").environ.get("MRAGAN_PACK_AT_START") is not None


class ImagePool():
    """cycle_gan_model.py:8-35: history of generated images (Python `random`, like the
    reference).  Returns the batch as one tensor (torch.cat of the chosen images)."""

    def __init__(self, pool_size):
        self.pool_size = pool_size
        if self.pool_size > 0:
            self.num_imgs = 0
            self.images = []

    def query(self, images):
        if self.pool_size == 0:
            return images
        out = []
        for image in images:
            image = image.detach().unsqueeze(0)
            if self.num_imgs < self.pool_size:
                self.num_imgs += 1
                self.images.append(image)
                out.append(image)
            else:
                if random.uniform(0, 1) > 0.5:
                    rid = random.randint(0, self.pool_size - 1)
                    tmp = self.images[rid].clone()
                    self.images[rid] = image
                    out.append(tmp)
                else:
                    out.append(image)
        return torch.cat(out, 0)


class DeviceImagePool:
    """ImagePool.query as a device-side index plan, for the fused (and graph-replayed) step.

    `plan()` makes exactly the reference's draws (`random.uniform`, then `random.randint` for a
    swap; cycle_gan_model.py:20-35) on the host and resolves them into two index vectors;
    `apply()` executes them on the device.  The pool's rows live in one tensor
    [P slots | trash | fakes of this batch (capacity ≥ b)]: the returned batch is an index_select
    (a slot's old image, or a fake), the stores an index_copy of the fakes into the slots that end
    up holding them (the others go to the trash row).  Same images, same order as ImagePool, for
    any sequence of batch sizes (the last, smaller batch of an epoch included: train.py:52 has no
    drop_last) — the slot rows never move when the fake region grows."""

    def __init__(self, pool_size):
        self.pool_size = pool_size
        self.num_imgs = 0
        self.buf = None

    def plan(self, b):
        """Host draws for a batch of b fakes → (ret[b], store[b]) row indices into `buf`."""
        P = self.pool_size
        ret, holder = [], {}
        for k in range(b):
            if P == 0:
                ret.append(P + 1 + k)
            elif self.num_imgs < P:
                holder[self.num_imgs] = k
                self.num_imgs += 1
                ret.append(P + 1 + k)
            elif random.uniform(0, 1) > 0.5:
                rid = random.randint(0, P - 1)
                ret.append(P + 1 + holder[rid] if rid in holder else rid)
                holder[rid] = k
            else:
                ret.append(P + 1 + k)
        store = [P] * b
        for slot, k in holder.items():
            store[k] = slot
        return ret, store

    def reserve(self, b, image_shape, device, dtype=torch.float32):
        """Make room for a batch of b images of `image_shape`; stored images are kept.  Called on
        the host before the step (a graph capture must not allocate or move the pool)."""
        P = self.pool_size
        image_shape = tuple(image_shape)
        if self.buf is not None and (tuple(self.buf.shape[1:]) != image_shape or self.buf.device != device):
            if self.num_imgs:
                raise RuntimeError("DeviceImagePool: image shape changed with images in the pool")
            self.buf = None
        if self.buf is None or self.buf.shape[0] < P + 1 + b:
            nb = torch.zeros((P + 1 + b,) + image_shape, device=device, dtype=dtype)
            if self.buf is not None:
                nb[:P + 1].copy_(self.buf[:P + 1])
            self.buf = nb
        return self.buf

    def apply(self, fakes, out, ret_idx, store_idx):
        """fakes [b, ...] → out [b, ...]; ret_idx/store_idx: int64 index tensors from plan()."""
        P, b = self.pool_size, fakes.shape[0]
        buf = self.reserve(b, fakes.shape[1:], fakes.device, fakes.dtype)[:P + 1 + b]
        buf[P + 1:].copy_(fakes)
        torch.index_select(buf, 0, ret_idx, out=out)
        buf.index_copy_(0, store_idx, fakes)

    def query(self, images):
        """The reference's `ImagePool.query` (cycle_gan_model.py:15-35) on a device batch
        [b, C, D, H, W]: returns the pooled batch as one tensor, same draws, same images."""
        if self.pool_size == 0:
            return images
        b = images.shape[0]
        ret, store = self.plan(b)
        x = images.detach().float().permute(0, 2, 3, 4, 1).contiguous()
        out = torch.empty_like(x)
        dev = x.device
        self.apply(x, out, torch.tensor(ret, dtype=torch.int64, device=dev),
                   torch.tensor(store, dtype=torch.int64, device=dev))
        return out.permute(0, 4, 1, 2, 3)


class _Lanes:
    """Two in-order lanes for the step's independent chains: lane 0 is the current stream,
    lane 1 an auxiliary stream forked from it (under capture: two branches of the HIP graph).
    `on(i)` issues on lane i with lane i's workspace; `mark` / `wait` order one lane after a
    point of the other; `join` ends the fork.  With `parallel=False` both lanes are the current
    stream (the --single_stream order, also what bench.py times kernels under)."""

    def __init__(self, aux, parallel=True):
        from mragan_hip import ops
        self._ops = ops
        cur = torch.cuda.current_stream()
        if ops.in_tickets_enabled():
            # the ticket pool's zero-fill must precede both lanes' first ticket draw
            ops.ensure_ticket_pool(cur.device)
        self.s = [cur, aux if parallel else cur]
        self.parallel = parallel
        if parallel:
            aux.wait_stream(cur)

    def on(self, i):
        lanes = self

        class _On:
            def __enter__(self_):
                self_.st = torch.cuda.stream(lanes.s[i])
                self_.ln = lanes._ops.lane(i)
                self_.st.__enter__()
                self_.ln.__enter__()

            def __exit__(self_, *exc):
                self_.ln.__exit__(*exc)
                self_.st.__exit__(*exc)
                return False
        return _On()

    def mark(self, i):
        ev = torch.cuda.Event()
        ev.record(self.s[i])
        return ev

    def wait(self, i, ev):
        if self.parallel:
            self.s[i].wait_event(ev)

    def join(self):
        if self.parallel:
            self.s[0].wait_stream(self.s[1])


class _SideLanes:
    """Two more in-order streams forked from the current (origin) stream and joined back to it,
    with workspace lanes 2 and 3: the D phase beside the G backward (which holds lanes 0 and 1).
    Only origin ↔ side edges (fork: each side stream waits for the origin; join: the origin waits
    for each) — the capture topology this ROCm accepts."""

    def __init__(self, streams):
        from mragan_hip import ops
        self._ops = ops
        cur = torch.cuda.current_stream()
        self.cur = cur
        self.s = list(streams)
        for st in self.s:
            st.wait_stream(cur)

    def on(self, i):
        lanes = self

        class _On:
            def __enter__(self_):
                self_.st = torch.cuda.stream(lanes.s[i])
                self_.ln = lanes._ops.lane(2 + i)
                self_.st.__enter__()
                self_.ln.__enter__()

            def __exit__(self_, *exc):
                self_.ln.__exit__(*exc)
                self_.st.__exit__(*exc)
                return False
        return _On()

    def mark(self, i):
        ev = torch.cuda.Event()
        ev.record(self.s[i])
        return ev

    def join(self):
        for st in self.s:
            self.cur.wait_stream(st)


def _to_ndhwc(x: torch.Tensor) -> torch.Tensor:
    return x.float().permute(0, 2, 3, 4, 1).contiguous()


def _to_ncdhw(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 4, 1, 2, 3)


def ops_mod():
    from mragan_hip import ops
    return ops


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics (amsgrad=False, weight_decay=0) as one HIP kernel per flat
    parameter buffer.  Subclasses torch.optim.Optimizer so LambdaLR & co. drive `lr`."""

    def __init__(self, nets, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.nets = list(nets)
        params = list(itertools.chain(*[n.parameters() for n in self.nets]))
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=False))
        self._m = {}
        self._v = {}
        self.step_count = 0
        self.grad_scale = 1.0
        # loss-scaled (fp16) training: skip the update of a step whose gradients overflowed, like
        # torch.cuda.amp.GradScaler.step (device flag, graph-replayable; count in `skipped()`)
        self.check_finite = False
        self._flag = None
        self._skipped = None

    def zero_grad(self, set_to_none: bool = True):
        from mragan_hip import ops
        for n in self.nets:
            networks3D.ensure_flat(n)
            ops.fill(n._flat_grad, 0.0)

    def advance(self):
        """Host half of a step: bump the step count and return the six values step_dev reads — the
        kernel's scalars, or with check_finite the base {lr, beta1, beta2, eps, step, grad_scale}
        that step_dev turns into them on the device net of the skipped steps (mragan_adam_rebias:
        like GradScaler, a skipped update does not advance the bias corrections)."""
        self.step_count += 1
        g = self.param_groups[0]
        beta1, beta2 = g['betas']
        if self.check_finite:
            return [float(g['lr']), float(beta1), float(beta2), float(g['eps']), float(self.step_count),
                    float(self.grad_scale)]
        return ops_mod().adam_hyper(g['lr'], beta1, beta2, g['eps'], self.step_count, self.grad_scale)

    def _state(self, n):
        key = id(n)
        if key not in self._m or self._m[key].numel() != n._flat_param.numel():
            self._m[key] = torch.zeros_like(n._flat_param)
            self._v[key] = torch.zeros_like(n._flat_param)
        return self._m[key], self._v[key]

    @torch.no_grad()
    def step_dev(self, hyper):
        """Device half: one fused Adam kernel per flat buffer with the scalars in `hyper`
        (written by the host before the kernels run; graph-replayable)."""
        ops = ops_mod()
        if self.check_finite:
            if self._flag is None:
                dev = self.nets[0]._flat_grad.device
                self._flag = torch.zeros(1, dtype=torch.int32, device=dev)
                self._skipped = torch.zeros(1, dtype=torch.int32, device=dev)
                self._hyper = torch.empty(6, dtype=torch.float32, device=dev)
            ops.adam_rebias(hyper, self._skipped, self._hyper)     # `hyper` holds advance()'s base
            hyper = self._hyper
            for n in self.nets:
                networks3D.ensure_flat(n)
                ops.nonfinite_flag(n._flat_grad, self._flag)
        for n in self.nets:
            networks3D.ensure_flat(n)
            m, v = self._state(n)
            if self.check_finite:
                ops.adam_dev_checked(n._flat_param, n._flat_grad, m, v, hyper, self._flag)
            else:
                ops.adam_dev(n._flat_param, n._flat_grad, m, v, hyper)
            n.mark_params_dirty()
        if self.check_finite:
            ops.skip_count(self._flag, self._skipped)
        # what torch's step wrapper records for an LR scheduler (it warns otherwise)
        self._opt_called = True

    @torch.no_grad()
    def step_net(self, n, hyper):
        """step_dev for one of the optimizer's networks (no found-inf check: its flag spans every
        network).  The overlapped single-GPU step issues each network's update at the end of the
        stream that finished its gradients (CycleGANModel._phase_GD)."""
        assert not self.check_finite, "step_net: the found-inf check needs every network's gradients"
        networks3D.ensure_flat(n)
        m, v = self._state(n)
        ops_mod().adam_dev(n._flat_param, n._flat_grad, m, v, hyper)
        n.mark_params_dirty()
        self._opt_called = True

    def skipped(self) -> int:
        """Steps whose update was skipped for a non-finite gradient (synchronizes)."""
        return 0 if self._skipped is None else int(self._skipped.item())

    @torch.no_grad()
    def step(self, closure=None):
        from mragan_hip import ops
        self.step_count += 1
        g = self.param_groups[0]
        beta1, beta2 = g['betas']
        for n in self.nets:
            networks3D.ensure_flat(n)
            key = id(n)
            if key not in self._m or self._m[key].numel() != n._flat_param.numel():
                self._m[key] = torch.zeros_like(n._flat_param)
                self._v[key] = torch.zeros_like(n._flat_param)
            ops.adam(n._flat_param, n._flat_grad, self._m[key], self._v[key], g['lr'], beta1, beta2, g['eps'],
                     self.step_count, self.grad_scale)
            n.mark_params_dirty()
        self._opt_called = True


class CycleGANModel(BaseModel):
    def name(self):
        return 'CycleGANModel'

    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        parser.set_defaults(no_dropout=True)
        if is_train:
            parser.add_argument('--lambda_A', type=float, default=10.0, help='weight for cycle loss (A -> B -> A)')
            parser.add_argument('--lambda_B', type=float, default=10.0, help='weight for cycle loss (B -> A -> B)')
            parser.add_argument('--lambda_identity', type=float, default=0.5,
                                help='weight of the identity mapping loss, relative to the reconstruction loss')
            parser.add_argument('--lambda_co_A', type=float, default=2,
                                help='weight for correlation coefficient loss (A -> B)')
            parser.add_argument('--lambda_co_B', type=float, default=2,
                                help='weight for correlation coefficient loss (B -> A )')
        return parser

    def initialize(self, opt):
        BaseModel.initialize(self, opt)
        from mragan_hip import ops
        self.precision = getattr(opt, 'conv_precision', 'f32')
        ops.set_conv_precision(self.precision)
        # fp16 operands: gradients are computed scaled (static loss scale) and unscaled by Adam;
        # p.grad then holds loss_scale × the gradient (like torch.amp before unscale_)
        self.loss_scale = float(getattr(opt, 'loss_scale', 1024.0)) if self.precision == 'fp16' else 1.0
        ops.set_loss_scale(self.loss_scale)
        self.loss_names = ['D_A', 'G_A', 'cycle_A', 'idt_A', 'D_B', 'G_B', 'cycle_B', 'idt_B']
        visual_names_A = ['real_A', 'fake_B', 'rec_A']
        visual_names_B = ['real_B', 'fake_A', 'rec_B']
        if self.isTrain and self.opt.lambda_identity > 0.0:
            visual_names_A.append('idt_A')
            visual_names_B.append('idt_B')
        self.visual_names = visual_names_A + visual_names_B
        self.model_names = ['G_A', 'G_B', 'D_A', 'D_B'] if self.isTrain else ['G_A', 'G_B']

        self.netG_A = networks3D.define_G(opt.input_nc, opt.output_nc, opt.ngf, opt.netG, opt.norm,
                                          not opt.no_dropout, opt.init_type, opt.init_gain, self.gpu_ids)
        self.netG_B = networks3D.define_G(opt.output_nc, opt.input_nc, opt.ngf, opt.netG, opt.norm,
                                          not opt.no_dropout, opt.init_type, opt.init_gain, self.gpu_ids)
        if self.isTrain:
            use_sigmoid = opt.no_lsgan
            self.netD_A = networks3D.define_D(opt.output_nc, opt.ndf, opt.netD, opt.n_layers_D, opt.norm, use_sigmoid,
                                              opt.init_type, opt.init_gain, self.gpu_ids)
            self.netD_B = networks3D.define_D(opt.input_nc, opt.ndf, opt.netD, opt.n_layers_D, opt.norm, use_sigmoid,
                                              opt.init_type, opt.init_gain, self.gpu_ids)
            self.fake_A_pool = DeviceImagePool(opt.pool_size)
            self.fake_B_pool = DeviceImagePool(opt.pool_size)
            self.use_lsgan = not opt.no_lsgan
            self.criterionGAN = networks3D.GANLoss(use_lsgan=self.use_lsgan).to(self.device)
            self.criterionCycle = torch.nn.L1Loss()
            self.criterionIdt = torch.nn.L1Loss()
            self.optimizer_G = FusedAdam([self.netG_A, self.netG_B], lr=opt.lr, betas=(opt.beta1, 0.999))
            self.optimizer_D = FusedAdam([self.netD_A, self.netD_B], lr=opt.lr, betas=(opt.beta1, 0.999))
            self.optimizers = [self.optimizer_G, self.optimizer_D]
            self.optimizer_G.check_finite = self.optimizer_D.check_finite = self.loss_scale != 1.0
            self._loss_buf = torch.zeros(8, device=self.device, dtype=torch.float32)
            for i, n in enumerate(self.loss_names):
                setattr(self, 'loss_' + n, self._loss_buf[i])
        self._dist = None
        self._use_graph = self.isTrain and not getattr(opt, 'no_cuda_graph', False) and self.device.type == 'cuda'
        self.parallel_lanes = not getattr(opt, 'single_stream', False)
        self._aux_stream = None
        self._d_streams = None          # the D phase's two streams beside the G backward (_phase_GD)
        self._graphs = None          # (G-phase graph, D-phase graph) of the step being replayed
        self._rs_tables = None       # running-stat update tables of that capture
        self._graph_key = None
        self._graph_cache = OrderedDict()   # capture key → captured step (LRU, GRAPH_CACHE entries)
        self._eager_steps = 0
        self._eager_shapes = set()   # input shapes stepped eagerly (workspaces sized for them)
        self._in = {}                # persistent input buffers (the graphs read them)

    # ------------------------------------------------------------------ inputs / visuals
    def set_input(self, input):
        AtoB = self.opt.which_direction == 'AtoB'
        self.real_A = self._stage_input('A', input[0 if AtoB else 1])
        self.real_B = self._stage_input('B', input[1 if AtoB else 0])

    def _stage_input(self, key, x):
        """Copy into a persistent device buffer per input shape (same values; a captured step reads
        it, and alternating batch shapes keep their buffers — and their cached captures)."""
        k = (key, tuple(x.shape), x.dtype)
        buf = self._in.get(k)
        if buf is None:
            buf = torch.empty(x.shape, dtype=x.dtype, device=self.device)
            self._in[k] = buf
        buf.copy_(x, non_blocking=True)
        return buf

    def _publish(self, **ndhwc):
        for k, v in ndhwc.items():
            setattr(self, k, _to_ncdhw(v))

    @property
    def loss_cor_coe_GA(self):      # computed-but-unused in the reference (cycle_gan_model.py:217)
        return networks3D.Cor_CoeLoss(self.fake_B, self.real_A) * self.opt.lambda_co_A

    @property
    def loss_cor_coe_GB(self):      # cycle_gan_model.py:218
        return networks3D.Cor_CoeLoss(self.fake_A, self.real_B) * self.opt.lambda_co_B

    # ------------------------------------------------------------------ plain forward (test)
    def forward(self):
        """cycle_gan_model.py:121-136 (used by test()): the four generator passes."""
        A, B = _to_ndhwc(self.real_A), _to_ndhwc(self.real_B)
        pGA, pGB = self.netG_A.plan, self.netG_B.plan
        from mragan_hip import engine
        c1 = pGA.forward(A)
        c2 = pGB.forward(c1.out)
        c3 = pGB.forward(B)
        c4 = pGA.forward(c3.out)
        keep = [engine.apply_running_updates(pGA.running_entries([(c1, 0, c1.N), (c4, 0, c4.N)]), A.device),
                engine.apply_running_updates(pGB.running_entries([(c2, 0, c2.N), (c3, 0, c3.N)]), A.device)]
        self._publish(fake_B=c1.out, rec_A=c2.out, fake_A=c3.out, rec_B=c4.out)
        del keep

    # ------------------------------------------------------------------ training step
    def forward_train(self):
        """The four cycle passes plus the two identity passes, batched (see module doc).  With
        lambda_identity <= 0 the reference runs no identity pass (cycle_gan_model.py:174-194),
        so each generator then runs its own input only."""
        for n in (self.netG_A, self.netG_B, self.netD_A, self.netD_B):
            networks3D.ensure_flat(n)
        A, B = _to_ndhwc(self.real_A), _to_ndhwc(self.real_B)
        b = A.shape[0]
        self._A, self._B, self._b = A, B, b
        self._idt = self.opt.lambda_identity > 0
        pGA, pGB = self.netG_A.plan, self.netG_B.plan
        # each lane packs the networks it runs first (G_A, D_A on lane 0; G_B, D_B on lane 1) and
        # waits for the other lane's generator pack only before its cycle pass: the four repacks
        # no longer run serially ahead of the fork
        ln = self._lanes()
        # the discriminators are first used on the side streams in the overlapped schedule: their
        # repacks run there (backward_G), off the lanes' critical start
        d_here = not (self._overlap_D() and not _FROZEN_D_ON_LANES)
        with ln.on(0):
            pGA.ensure_packed()
            if d_here:
                self.netD_A.plan.ensure_packed()
            packed_0 = ln.mark(0)
        with ln.on(1):
            pGB.ensure_packed()
            if d_here:
                self.netD_B.plan.ensure_packed()
            packed_1 = ln.mark(1)
        with ln.on(0):          # lane 0: G_A(real_A) → G_B(fake_B)
            self._cGA1 = pGA.forward(torch.cat([A, B], 0) if self._idt else A)   # [fake_B; idt_A]
            fake_B = self._cGA1.out[:b]
            ln.wait(0, packed_1)
            self._cGB2 = pGB.forward(fake_B)                     # rec_A
        with ln.on(1):          # lane 1: G_B(real_B) → G_A(fake_A)
            self._cGB1 = pGB.forward(torch.cat([B, A], 0) if self._idt else B)   # [fake_A; idt_B]
            fake_A = self._cGB1.out[:b]
            ln.wait(1, packed_0)
            self._cGA2 = pGA.forward(fake_A)                     # rec_B
        ln.join()
        self._fake_B, self._fake_A = fake_B, fake_A
        self._publish(fake_B=fake_B, fake_A=fake_A, rec_A=self._cGB2.out, rec_B=self._cGA2.out)
        if self._idt:
            self._publish(idt_A=self._cGA1.out[b:], idt_B=self._cGB1.out[b:])

    def backward_G(self, side=None):
        """cycle_gan_model.py:163-225: identity, GAN and cycle losses; backward through the 6
        generator passes and (data gradient only) the 2 frozen discriminator passes.

        The GAN losses' data gradients (D_A(fake_B) → d fake_B, D_B(fake_A) → d fake_A) feed only
        the first-pass backwards, not the cycle-pass ones: each frozen discriminator writes its
        data gradient into its own buffer (dD_A / dD_B), and the first passes take the two sources
        [lane's gradient, D's] — summed in the head's tanh backward (fake half: cycle + GAN;
        identity half: identity + 0).  With `side` (_SideLanes, the single-GPU overlapped
        schedule, _phase_GD) the frozen passes, and after them the D phase, run on the two side
        streams beside the cycle-pass backwards, and the origin (lane 0) waits for both frozen
        passes before its first-pass backward (lane 1 waits for the origin there as before);
        without it they run on the lanes ahead of the cycle passes.  Every schedule forms the same
        sums in the same order: the results are bit-identical (tests/test_graph_gpu.py).

        Lane 0 runs loss_cycle_A / loss_idt_A and then G_B's rec_A pass (G_B weight gradients +
        d fake_B), lane 1 the mirror image.  The cycle passes leave their ResnetBlock
        weight-gradient operands (planes) to the first passes of the same generator on the other
        lane, which run each conv's weight gradient once over both passes' instances
        (NetPlan.backward wgrad_defer / wgrad_pair); those tensors stay referenced until the lanes
        are joined."""
        from mragan_hip import ops
        b, A, B = self._b, self._A, self._B
        lA, lB, li = self.opt.lambda_A, self.opt.lambda_B, self.opt.lambda_identity
        L = self._loss_buf
        pDA, pDB = self.netD_A.plan, self.netD_B.plan
        pGA, pGB = self.netG_A.plan, self.netG_B.plan
        # allocated before the fork: both lanes' tensors outlive it
        dGA1 = torch.empty_like(self._cGA1.out)     # d/d[fake_B; idt_A]: cycle + identity losses
        dGB1 = torch.empty_like(self._cGB1.out)     # d/d[fake_A; idt_B]
        dDA = torch.empty_like(dGA1)                # d/d[fake_B; idt_A]: D_A's GAN loss (0 on idt_A)
        dDB = torch.empty_like(dGB1)
        d_recA = torch.empty_like(self._cGB2.out)
        d_recB = torch.empty_like(self._cGA2.out)
        if not self._idt:                                                              # reference: 0
            ops.fill(L[3:4], 0.0)
            ops.fill(L[7:8], 0.0)

        def frozen(pD, fake, slot, dD):
            cD = pD.forward(fake)
            dlog = torch.empty_like(cD.out)
            ops.gan_loss(cD.out, 1.0, self.use_lsgan, 1.0, L[slot:slot + 1], dlog)
            pD.backward(cD, [dlog], need_wgrad=False, need_input_grad=True, dx_out=dD[:b])
            if self._idt:
                ops.fill(dD[b:], 0.0)
            return cD

        def l1s(rec, real_rec, lam, d_rec, cG1, dG1, real_idt, lam_idt, idt_slot, cyc_slot):
            ops.l1_loss(rec, real_rec, lam, L[cyc_slot:cyc_slot + 1], d_rec)
            if self._idt:
                ops.l1_loss(cG1.out[b:], real_idt, lam_idt, L[idt_slot:idt_slot + 1], dG1[b:])

        if side is not None:
            adam_in = self._adam_in_lanes()
            with side.on(0):
                pDA.ensure_packed()
                self._cDA1 = frozen(pDA, self._fake_B, 1, dDA)
                d_done_A = side.mark(0)
                self.backward_D_A()
                if adam_in:     # D_A's parameters are read on this stream only
                    self.optimizer_D.step_net(self.netD_A, self._step_hyper[6:12])
            with side.on(1):
                pDB.ensure_packed()
                self._cDB1 = frozen(pDB, self._fake_A, 5, dDB)
                d_done_B = side.mark(1)
                self.backward_D_B()
                if adam_in:
                    self.optimizer_D.step_net(self.netD_B, self._step_hyper[6:12])
        ln = self._lanes()
        defer_A, defer_B = {}, {}
        with ln.on(0):
            if side is None:
                self._cDA1 = frozen(pDA, self._fake_B, 1, dDA)
            l1s(self._cGB2.out, A, lA, d_recA, self._cGA1, dGA1, B, lB * li, 3, 2)
            pGB.backward(self._cGB2, [d_recA], need_input_grad=True, dx_out=dGA1[:b], wgrad_defer=defer_B)
            if side is not None:
                cur = torch.cuda.current_stream()
                cur.wait_event(d_done_A)            # origin ← side joins (the frozen passes)
                cur.wait_event(d_done_B)
            rec_done_0 = ln.mark(0)                 # lane 1 waits this: d fake_A complete too
        with ln.on(1):
            if side is None:
                self._cDB1 = frozen(pDB, self._fake_A, 5, dDB)
            l1s(self._cGA2.out, B, lB, d_recB, self._cGB1, dGB1, A, lA * li, 7, 6)
            pGA.backward(self._cGA2, [d_recB], need_input_grad=True, dx_out=dGB1[:b], wgrad_defer=defer_A)
            rec_done_1 = ln.mark(1)
        keep = (list(defer_A.values()), list(defer_B.values()))
        adam_in = side is not None and self._adam_in_lanes()
        tail = adam_in and self._pack_tail()
        with ln.on(0):
            ln.wait(0, rec_done_1)
            pGA.backward(self._cGA1, [dGA1, dDA], wgrad_pair=defer_A)
            if adam_in:         # every G_A gradient is done here (lane 1's G_A cycle pass is waited for)
                self.optimizer_G.step_net(self.netG_A, self._step_hyper[0:6])
                if tail:        # the next step's packs, at this lane's tail instead of its next start
                    pGA.ensure_packed()
        with ln.on(1):
            ln.wait(1, rec_done_0)
            pGB.backward(self._cGB1, [dGB1, dDB], wgrad_pair=defer_B)
            if adam_in:
                self.optimizer_G.step_net(self.netG_B, self._step_hyper[0:6])
                if tail:
                    pGB.ensure_packed()
        ln.join()
        del keep

    def _pack_tail(self):
        """The generators' weights are repacked right after their Adam update, at the end of their
        lanes (the overlapped single-GPU schedule with the updates inside it): the next step's lanes
        start with their forwards, and a graph replay leaves the generator packs fresh (the host's
        dirty flag stays clear; a parameter change from outside the step sets it, and the next step
        then repacks before its replay)."""
        return self._overlap_D() and self._adam_in_lanes() and not _PACK_AT_START

    def _lanes(self):
        if self.parallel_lanes and self._aux_stream is None:
            self._aux_stream = torch.cuda.Stream(device=self.device)
        return _Lanes(self._aux_stream, self.parallel_lanes)

    def backward_D_basic(self, netD, real, pool, fakes, ret_idx, store_idx, loss_slot):
        """cycle_gan_model.py:138-149 with real and (pooled, detached) fake batched."""
        from mragan_hip import ops
        b = real.shape[0]
        plan = netD.plan
        x = torch.empty((2 * b,) + tuple(real.shape[1:]), device=real.device, dtype=torch.float32)
        x[:b].copy_(real)
        pool.apply(fakes, x[b:], ret_idx, store_idx)
        ctx = plan.forward(x)
        dlog = torch.empty_like(ctx.out)
        ops.gan_loss(ctx.out[:b], 1.0, self.use_lsgan, 0.5, loss_slot, dlog[:b])
        ops.gan_loss(ctx.out[b:], 0.0, self.use_lsgan, 0.5, loss_slot, dlog[b:], loss_accumulate=True)
        plan.backward(ctx, [dlog], need_wgrad=True, need_input_grad=False)
        return ctx

    def backward_D_A(self):
        i = self._step_idx
        self._cDA2 = self.backward_D_basic(self.netD_A, self._B, self.fake_B_pool, self._fake_B, i[0], i[1],
                                           self._loss_buf[0:1])

    def backward_D_B(self):
        i = self._step_idx
        self._cDB2 = self.backward_D_basic(self.netD_B, self._A, self.fake_A_pool, self._fake_A, i[2], i[3],
                                           self._loss_buf[4:5])

    def _running_entries(self):
        """Per network, the IN running-stat updates of this step in the reference's call order."""
        b = self._b
        idA = [(self._cGA1, b, b)] if self._idt else []     # idt_A = G_A(real_B), backward_G
        idB = [(self._cGB1, b, b)] if self._idt else []     # idt_B = G_B(real_A)
        return [self.netG_A.plan.running_entries([(self._cGA1, 0, b), (self._cGA2, 0, b)] + idA),
                self.netG_B.plan.running_entries([(self._cGB2, 0, b), (self._cGB1, 0, b)] + idB),
                self.netD_A.plan.running_entries([(self._cDA1, 0, b), (self._cDA2, 0, b), (self._cDA2, b, b)]),
                self.netD_B.plan.running_entries([(self._cDB1, 0, b), (self._cDB2, 0, b), (self._cDB2, b, b)])]

    def _running_stats(self):
        """Eager step: build the tables (pointers into this step's tensors) and launch."""
        from mragan_hip import engine
        self._keep = [engine.apply_running_updates(e, self._A.device) for e in self._running_entries()]

    def _running_stats_graphed(self):
        """Replayed step: the captured tensors are replay-stable, so the tables are built once
        per capture and the four small update kernels are launched after the D-phase replay."""
        from mragan_hip import engine
        if self._rs_tables is None:
            self._rs_tables = [(engine.running_table(e, self._A.device), len(e)) for e in self._running_entries() if e]
        for tab, n in self._rs_tables:
            engine.launch_running_update(tab, n)

    # ------------------------------------------------------------------ the step
    def _prepare_step(self):
        """Host half of a step: both pools' draws (reference order: fake_B_pool, then
        fake_A_pool) and both Adam steps' scalars, shipped to device buffers that the kernels
        (eager or replayed) read.  Returns nothing; the device buffers are persistent."""
        b = self.real_A.shape[0]
        retB, stB = self.fake_B_pool.plan(b)
        retA, stA = self.fake_A_pool.plan(b)
        sp = tuple(self.real_A.shape[2:])
        self.fake_B_pool.reserve(b, sp + (self.opt.output_nc,), self.real_A.device)
        self.fake_A_pool.reserve(b, sp + (self.opt.input_nc,), self.real_A.device)
        hyp = self.optimizer_G.advance() + self.optimizer_D.advance()
        idx = torch.tensor([retB, stB, retA, stA], dtype=torch.int64).pin_memory()
        hyp = torch.tensor(hyp, dtype=torch.float32).pin_memory()
        # one persistent index buffer per batch size (a captured step reads it: alternating batch
        # sizes keep their buffers and so their cached captures)
        if not hasattr(self, '_step_idx_bufs'):
            self._step_idx_bufs = {}
            self._step_hyper = torch.empty(12, dtype=torch.float32, device=self.device)
        self._step_idx = self._step_idx_bufs.get(tuple(idx.shape))
        if self._step_idx is None:
            self._step_idx = torch.empty(idx.shape, dtype=torch.int64, device=self.device)
            self._step_idx_bufs[tuple(idx.shape)] = self._step_idx
        self._step_idx.copy_(idx, non_blocking=True)
        self._step_hyper.copy_(hyp, non_blocking=True)

    def _phase_G(self):
        self.forward_train()
        self.set_requires_grad([self.netD_A, self.netD_B], False)
        self.optimizer_G.zero_grad()
        self.backward_G()

    def _overlap_D(self):
        """Single GPU with two lanes: the D phase runs beside the G backward (round 6)."""
        return self.parallel_lanes and not self._dist and not _TWO_PHASE

    def _adam_in_lanes(self):
        """In the overlapped schedule without a loss scale (no found-inf check spanning both
        networks of an optimizer): each network's Adam update runs at the end of the stream that
        completed its gradients, inside the step — D_A / D_B beside the G backward, G_A / G_B as
        each lane finishes — instead of four launches after it.  Same kernel, same operands."""
        return (self._overlap_D() and not _ADAM_AFTER and not self.optimizer_G.check_finite
                and not self.optimizer_D.check_finite and not _FROZEN_D_ON_LANES)

    def _phase_GD(self):
        """G phase and D phase in one: the D phase needs only the fakes (made by the G forwards) and
        the pre-update D weights — the reference's order (cycle_gan_model.py:227-240: G step, then D
        step on the same fakes) is kept exactly, since no D weight changes before the D Adam and the
        D gradients are written only by the D phase — so once the forwards are joined it runs on two
        more streams (D_A, D_B) forked from the origin, beside the G backward on lanes 0 / 1, and is
        joined at the end.  Its small, latency-bound launches fill CU slots the G backward leaves
        idle.  Same kernels on the same operands as _phase_G then _phase_D: bit-identical results."""
        self.forward_train()
        self.set_requires_grad([self.netD_A, self.netD_B], False)
        self.optimizer_G.zero_grad()
        self.optimizer_D.zero_grad()
        if self._d_streams is None:
            self._d_streams = (torch.cuda.Stream(device=self.device), torch.cuda.Stream(device=self.device))
        side = _SideLanes(self._d_streams)
        if _FROZEN_D_ON_LANES:
            with side.on(0):
                self.backward_D_A()
            with side.on(1):
                self.backward_D_B()
            self.backward_G()
        else:
            self.backward_G(side)                   # the frozen D passes and the D phase on `side`
        side.join()
        if not torch.cuda.is_current_stream_capturing():
            self._running_stats()

    def _phase_D(self):
        self.set_requires_grad([self.netD_A, self.netD_B], True)
        self.optimizer_D.zero_grad()
        ln = self._lanes()
        with ln.on(0):
            self.backward_D_A()
        with ln.on(1):
            self.backward_D_B()
        ln.join()
        if not torch.cuda.is_current_stream_capturing():
            self._running_stats()

    def _capture_key(self):
        nets = (self.netG_A, self.netG_B, self.netD_A, self.netD_B)
        return (tuple(self.real_A.shape), tuple(self.real_B.shape), self.real_A.data_ptr(), self.real_B.data_ptr(),
                self.fake_A_pool.buf.data_ptr(), self.fake_B_pool.buf.data_ptr(),
                tuple(n._flat_param.data_ptr() for n in nets), tuple(n._flat_grad.data_ptr() for n in nets),
                self._step_idx.data_ptr(), self._step_hyper.data_ptr(), bool(self._dist))

    # attributes a captured step's tensors live in (re-published when a cached capture replays)
    _CAPTURE_ATTRS = ('_cGA1', '_cGA2', '_cGB1', '_cGB2', '_cDA1', '_cDA2', '_cDB1', '_cDB2', '_fake_A', '_fake_B',
                      '_A', '_B', '_b', '_idt', 'fake_A', 'fake_B', 'rec_A', 'rec_B', 'idt_A', 'idt_B')
    GRAPH_CACHE = 2          # the full batch and an epoch's smaller last batch

    def _use_capture(self):
        """Make the capture for the current key the replayed one: from the cache (alternating batch
        shapes — an epoch's smaller last batch — replay without recapturing), or a new
        capture (the least recently used one beyond GRAPH_CACHE entries is released)."""
        key = self._capture_key()
        if _NO_GRAPH_CACHE:
            self._graph_cache.clear()
        # a capture whose pool buffers were reallocated (a larger batch grew them) points at freed
        # memory: drop it (key fields 4, 5 are the pool buffers' addresses)
        for k in [k for k in self._graph_cache if k[4:6] != key[4:6]]:
            del self._graph_cache[k]
        ent = self._graph_cache.get(key)
        if ent is None:
            self._capture()
            from mragan_hip import engine
            self._rs_tables = [(engine.running_table(e, self._A.device), len(e)) for e in self._running_entries() if e]
            ent = dict(graphs=self._graphs, rs=self._rs_tables,
                       attrs={k: getattr(self, k) for k in self._CAPTURE_ATTRS if hasattr(self, k)})
            self._graph_cache[key] = ent
            while len(self._graph_cache) > self.GRAPH_CACHE:
                self._graph_cache.popitem(last=False)
        else:
            self._graph_cache.move_to_end(key)
            self._graphs, self._rs_tables = ent["graphs"], ent["rs"]
            for k, v in ent["attrs"].items():
                setattr(self, k, v)
        self._graph_key = key

    def _capture(self):
        """Record the G phase and the D phase as two HIP graphs (one memory pool).  Capturing
        launches nothing; the caller replays them for this step."""
        self._n_captures = getattr(self, '_n_captures', 0) + 1
        # the graphs must contain the weight repacks: the discriminators' (and, without the tail
        # repack, the generators') at the start of the step; with it the generators' are captured at
        # their lanes' tails and the step starts from the packs the previous step left
        tail = self._pack_tail()
        for n in (self.netG_A, self.netG_B, self.netD_A, self.netD_B):
            if tail and n in (self.netG_A, self.netG_B):
                n.plan.ensure_packed()
            else:
                n.mark_params_dirty()
        torch.cuda.synchronize()
        gG, gD = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        # thread_local: other threads (the process group's watchdog) may query the runtime
        # while this thread captures
        if self._overlap_D():
            with torch.cuda.graph(gG, stream=side, capture_error_mode="thread_local"):
                self._phase_GD()
            gD = None
        else:
            with torch.cuda.graph(gG, stream=side, capture_error_mode="thread_local"):
                self._phase_G()
            with torch.cuda.graph(gD, pool=gG.pool(), stream=side, capture_error_mode="thread_local"):
                self._phase_D()
        torch.cuda.current_stream().wait_stream(side)
        self._rs_tables = None
        self._graphs = (gG, gD)
        self._graph_key = self._capture_key()

    def optimize_parameters(self):
        """cycle_gan_model.py:227-240.  Single GPU: G phase, G Adam, D phase, D Adam (the
        reference's order up to the exact reordering below).  Data parallel: the G all-reduce
        overlaps the D phase (mragan_hip/dist.py) and both Adam steps follow it — exact, since
        the D phase reads only pre-update fakes and D weights.  From the second step on, both
        phases are replayed HIP graphs (captured once; `--no_cuda_graph` to disable)."""
        from mragan_hip.dist import GradSync, default_sync
        if self._dist is None:
            self._dist = default_sync() or False
            scale = 1.0 / (self._dist.world if self._dist else 1)
            self.optimizer_G.grad_scale = self.optimizer_D.grad_scale = scale / self.loss_scale
        from mragan_hip import ops
        ops.set_conv_precision(self.precision)      # process-wide: another model may have changed it
        ops.set_loss_scale(self.loss_scale)
        for n in (self.netG_A, self.netG_B, self.netD_A, self.netD_B):
            networks3D.ensure_flat(n)
        if self._dist:
            # one gradient buffer per optimizer (G_A + G_B, D_A + D_B): one all-reduce per phase
            self._grad_groups = (networks3D.group_grads([self.netG_A, self.netG_B]),
                                 networks3D.group_grads([self.netD_A, self.netD_B]))
        self._prepare_step()
        hG, hD = self._step_hyper[0:6], self._step_hyper[6:12]
        graphed = False
        shape_key = (tuple(self.real_A.shape), tuple(self.real_B.shape))
        # a shape is captured only after one eager step at it: that step grows the workspaces
        # (a capture must not allocate them)
        if self._use_graph and shape_key in self._eager_shapes:
            if self._graphs is None or self._graph_key != self._capture_key():
                self._use_capture()
            graphed = True
        if self._overlap_D():
            # one graph (or eager pass) for both phases, the D phase beside the G backward
            tail = self._pack_tail()
            if graphed:
                if tail:
                    # parameters changed since the last step (a load, a manual edit) mark the plan
                    # dirty: repack before the graph, which starts from the packs as they are
                    for n in (self.netG_A, self.netG_B):
                        n.plan.ensure_packed()
                self._graphs[0].replay()
                self._running_stats_graphed()
            else:
                self._phase_GD()
            if not self._adam_in_lanes():
                self.optimizer_G.step_dev(hG)
                self.optimizer_D.step_dev(hD)
            if graphed:
                for n in (self.netG_A, self.netG_B, self.netD_A, self.netD_B):
                    if not (tail and n in (self.netG_A, self.netG_B)):   # (the graph repacked those)
                        n.mark_params_dirty()
            else:
                self._eager_steps += 1
                self._eager_shapes.add(shape_key)
            return
        run_G = self._graphs[0].replay if graphed else self._phase_G
        run_D = self._graphs[1].replay if graphed else self._phase_D
        run_G()
        if graphed:
            run_D = lambda: (self._graphs[1].replay(), self._running_stats_graphed())
        if not self._dist:
            self.optimizer_G.step_dev(hG)
            run_D()
        else:
            sync_G = GradSync(self._dist.dist, self._dist.group)
            sync_G.start([self._grad_groups[0]])         # G_A + G_B: one collective
            run_D()
            sync_D = GradSync(self._dist.dist, self._dist.group)
            sync_D.start([self._grad_groups[1]])         # D_A + D_B
            sync_G.finish()
            self.optimizer_G.step_dev(hG)
            sync_D.finish()
        self.optimizer_D.step_dev(hD)
        if graphed:
            for n in (self.netG_A, self.netG_B, self.netD_A, self.netD_B):
                n.mark_params_dirty()
        else:
            self._eager_steps += 1
            self._eager_shapes.add(shape_key)
