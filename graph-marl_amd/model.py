"""NetMon and DQN on the HIP kernels (reference src/model.py, src/layernormlstm.py).

Parameter names match the reference's state_dicts (MLP.linear_layers.*,
nn.LSTMCell weight_ih/weight_hh/bias_ih/bias_hh, q_net.fc.*), so reference
checkpoints load unchanged. The forward arithmetic runs in libgraphmarl_amd:
  * gm_gemm_x3             every nn.Linear wider than 32 outputs (+ MLP leaky_relu): the
                           split-f16 MFMA form with fp32-order error (GM_GEMM=f32 or narrow
                           layers: gm_linear_f32, exact fp32 MFMA)
  * gm_lstm_pointwise      nn.LSTMCell gate math
  * gm_mp_aggregate        SimpleAggregation (sum / mean over I + A)
  * gm_netmon_readout      [h, last neighbour h] readout fused with the agent gather
Backward passes use the matching HIP backward kernels; weight/input gradients of
the dense layers use library GEMMs (torch.mm -> hipBLASLt).
"""
import ctypes as C
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L

SUM, MEAN = 0, 1

# --activation-function (src/main.py:194-197, 440-441: getattr(F, name), applied with its default
# arguments): the elementwise torch.nn.functional names, GM_ACT_* in include/graph_marl_amd.h. Codes up
# to softplus have a derivative that follows from the layer output; Z_ACTS need the pre-activation
# (their training forward keeps z and applies the activation with gm_act_fwd)
ACTIVATIONS = {"leaky_relu": 1, "relu": 2, "elu": 3, "tanh": 4, "sigmoid": 5, "relu6": 6, "hardtanh": 7,
               "hardsigmoid": 8, "selu": 9, "celu": 10, "softsign": 11, "logsigmoid": 12, "softplus": 13,
               "gelu": 14, "silu": 15, "mish": 16, "hardswish": 17, "tanhshrink": 18}
Z_ACTS = frozenset(range(14, 19))
# bias + activation epilogue code of gm_gemm_x3 / gm_gemm_f32 per activation code (GM_EPI_BIAS_ACT + act
# beyond the four named epilogues)
_EPI_OF_ACT = {0: 0, 1: 1, 2: 4, 3: 5, 4: 6, 5: 7}
GM_EPI_BIAS_ACT = 64


def act_code(activation):
    """GM_ACT_* code of an activation given by torch.nn.functional name (or function). Names that are
    not elementwise with default arguments (softmax, glu, rrelu's random slopes, ..) are refused."""
    if activation is None:
        return 0
    name = activation if isinstance(activation, str) else getattr(activation, "__name__", str(activation))
    name = {"log_sigmoid": "logsigmoid"}.get(name, name)  # F.logsigmoid.__name__
    if name not in ACTIVATIONS:
        raise NotImplementedError(f"--activation-function {name!r} is not built; the kernels provide "
                                  f"{', '.join(sorted(ACTIVATIONS))}")
    return ACTIVATIONS[name]


def epi_code(act):
    """gm_gemm epilogue code (GM_EPI_BIAS / GM_EPI_BIAS_<ACT> / GM_EPI_BIAS_ACT + act) of an activation code."""
    return _EPI_OF_ACT.get(act, GM_EPI_BIAS_ACT + act)


def act_fwd(z, act):
    """y = act(z) elementwise on the device (gm_act_fwd), z [rows, cols] contiguous."""
    y = torch.empty_like(z)
    L.check(L.lib().gm_act_fwd(z.data_ptr(), z.shape[0], z.shape[1], act, y.data_ptr(), _s()))
    return y


def _s():
    return L.stream_ptr()


def _pad_stride(k):
    return (k + 3) // 4 * 4


class _WeightCache:
    """fp32 weight with its row stride padded to a multiple of 4 (16-byte rows), and its
    split-f16 packing for gm_gemm_x3 (both refreshed when the parameter changes)."""

    def __init__(self):
        self.slots = {}  # form -> (key, value, L.Published): shared by streams (StreamedRollout groups)

    def __deepcopy__(self, memo):
        return _WeightCache()  # a copied module (target network) packs its own parameters

    def _get(self, form, key, build):
        k, v, pub = self.slots.get(form, (None, None, None))
        if k != key:
            v = build()
            self.slots[form] = (key, v, L.Published())
        else:
            pub.acquire(v)
        return v

    def x3(self, w):
        from . import fused as FU

        def build():
            wp, ldw = self.get(w)
            return FU.X3(wp, ldw, w.shape[0], w.shape[1])
        return self._get("x3", (w.data_ptr(), w._version), build)

    def x3t(self, w):
        """split-f16 packing of w^T ([in][out]) for the input-gradient GEMM gx = gy @ w."""
        from . import fused as FU

        def build():
            wt, ldt = FU._pad_cols(w.detach().t())
            return FU.X3(wt, ldt, w.shape[1], w.shape[0])
        return self._get("x3t", (w.data_ptr(), w._version), build)

    def get(self, w):
        n, k = w.shape
        kp = _pad_stride(k)
        if kp == k and w.is_contiguous():
            return w, k
        return self._get("pad", (w.data_ptr(), w._version, kp),
                         lambda: F.pad(w.detach(), (0, kp - k)).contiguous()), kp


def _x3_rows_ok(x2d, ldx, n):
    from . import fused as FU

    return FU.use_x3(n) and ldx % 4 == 0 and x2d.data_ptr() % 16 == 0


def _amax_slot(x2d, ldx, n, wanted):
    """Zeroed device slot for the forward GEMM to publish max|x| into (the weight gradient's
    operand scale, so backward needs no extra pass over x), or None."""
    if wanted and x2d.shape[0] >= 4096 and _x3_rows_ok(x2d, ldx, n):
        return torch.zeros(1, device=x2d.device)
    return None


def _finish_scale(slot):
    from . import fused as FU

    L.check(FU._setup().gm_absmax_finish(slot.data_ptr(), L.stream_ptr()))
    return slot


def linear_raw(x2d, ldx, k, w, b, act, out=None, ldy=None, wcache=None, tag=None, amax=None):
    """y = act(x @ w^T + b) on the MFMA kernel. x2d: row-major rows with stride ldx.
    amax: slot from _amax_slot (split-f16 form only; the kernel publishes max|x| into it)."""
    m = x2d.shape[0]
    n = w.shape[0]
    wp, ldw = (wcache.get(w) if wcache is not None else _WeightCache().get(w))
    if out is None:
        out = torch.empty(m, n, device=x2d.device, dtype=torch.float32)
        ldy = n
    from . import fused as FU

    if _x3_rows_ok(x2d, ldx, n):
        # split-f16 form (fp32-order error, tests/test_fused_gpu.py), as in the rollout
        x3 = (wcache if wcache is not None else _WeightCache()).x3(w)
        FU.gemm(FU.dense(x2d.data_ptr(), ldx, k, amax=None if amax is None else amax.data_ptr()), None,
                wp.data_ptr(), ldw, L.ptr(b), m, n, epi_code(act), out.data_ptr(), ldy,
                tag=tag and f"linear:{tag}:{m}x{n}x{k}", x3=x3)
        return out
    assert amax is None, "amax needs the split-f16 form"
    with L.timed(tag and f"linear:{tag}:{m}x{n}x{k}"):
        L.check(L.lib().gm_linear_f32(L.ptr(x2d), ldx, L.ptr(wp), ldw, L.ptr(b), m, n, k, act, L.ptr(out), ldy,
                                      _s()))
    return out


def _as_rows(x):
    """(2-D view, row stride, K) of a tensor whose last dim is contiguous."""
    k = x.shape[-1]
    x2 = x.reshape(-1, k) if x.dim() != 2 else x
    if x2.stride(-1) != 1 or (x2.stride(0) % 4) != 0 or (x2.data_ptr() % 16) != 0:
        x2 = F.pad(x2, (0, _pad_stride(k) - k)).contiguous()
        return x2, x2.stride(0), k
    return x2, x2.stride(0), k


def _gy_scale(gy):
    """Device power-of-two scale of a gradient operand (gm_absmax_scale), shared by its dgrad /
    wgrad GEMMs."""
    from . import fused as FU

    sc = torch.empty(1, device=gy.device)
    L.check(FU._setup().gm_absmax_scale(gy.data_ptr(), gy.numel(), sc.data_ptr(), L.stream_ptr()))
    return sc


def _dgrad(gy, w, wcache=None, sc=None):
    """gx = gy @ w. Split-f16 form over the packed w^T with gy scaled by a device power of two
    (gm_absmax_scale: gradients sit far below the range where both f16 pieces are normal);
    library fp32 GEMM when the shapes do not fit the kernel."""
    from . import fused as FU

    n, k = w.shape
    if FU.use_x3(k) and n % 4 == 0:
        gy = gy.contiguous()
        if gy.data_ptr() % 16 == 0:
            import ctypes as C

            lib = FU._setup()
            x3 = (wcache if wcache is not None else _WeightCache()).x3t(w)
            sc = _gy_scale(gy) if sc is None else sc
            gx = torch.empty(gy.shape[0], k, device=gy.device)
            # gm_gemm_x3_dgrad without a mask (split = k): its LDS-DMA tile at training sizes
            # (the sequence-batched update's input-gradient kernel), the register-staged one otherwise
            a = FU.dense(gy.data_ptr(), n, n, scale=sc.data_ptr())
            L.check(lib.gm_gemm_x3_dgrad(C.byref(a), x3.wp.data_ptr(), x3.sinv.data_ptr(), gy.shape[0], k, k, None,
                                         0, gx.data_ptr(), k, None, 0, None, None, _s()))
            return gx
    return gy @ w


def _wgrad(gy, x, k, sa=None, sb=None):
    """gW = gy^T @ x[:, :k], a reduction over the batch rows: split-K split-f16 GEMM on the
    K-major operands (gm_gemm_x3_wgrad; both scaled by device powers of two), partials summed
    here; library fp32 GEMM when the shapes do not fit the kernel."""
    from . import fused as FU

    Mb, o = gy.shape
    N = (k + 3) // 4 * 4
    ldx = x.stride(0)
    if not (FU.use_x3(k) and Mb >= 4096 and o % 4 == 0 and N <= ldx and ldx % 4 == 0 and x.stride(1) == 1
            and x.data_ptr() % 16 == 0):
        return gy.t() @ x[:, :k]
    gy = gy.contiguous()
    if gy.data_ptr() % 16:
        return gy.t() @ x[:, :k]
    lib = FU._setup()
    dev = gy.device
    sa = _gy_scale(gy) if sa is None else sa
    if sb is None:
        # scale from the k real columns; the up to 3 padding columns only reach output columns >= k
        sb = torch.empty(1, device=dev)
        L.check(lib.gm_absmax_scale_rows(x.data_ptr(), Mb, k, ldx, sb.data_ptr(), L.stream_ptr()))
    kchunk, splits = _wgrad_chunk(Mb, ((o + 127) // 128) * ((N + 127) // 128))
    part = torch.empty(splits, o, N, device=dev)
    L.check(lib.gm_gemm_x3_wgrad(gy.data_ptr(), o, x.data_ptr(), ldx, o, N, Mb, kchunk, sa.data_ptr(), sb.data_ptr(),
                                 part.data_ptr(), N, L.stream_ptr()))
    return part.sum(0)[:, :k]


def _wgrad_chunk(Mb, tiles, period=0):
    """Split-K plan of the weight-gradient kernel: (kchunk, splits). About 1024 blocks (two rounds of the 512
    resident 128 x 128 blocks; rounding the split count DOWN, so no partial third round), k chunks a multiple
    of the 32-deep k tile and, with a row map (period > 0), dividing the period."""
    splits = max(1, min(Mb // 2048, 1024 // max(1, tiles)))
    while splits > 1 and (tiles * splits) % 8:  # XCD-grouped chunks need tiles * splits % 8 == 0
        splits -= 1
    q = -(-(-(-Mb // splits)) // 32)  # ceil(ceil(Mb / splits) / 32)
    if period:
        if period % 32:
            return None, None
        while (period // 32) % q:
            q += 1
    kchunk = 32 * q
    return kchunk, -(-Mb // kchunk)


def _wgrad2(gy, srcs, sa):
    """Weight gradients gy^T @ x[:, :k] of one or two K-major sources that share the gradient operand gy, in ONE
    split-K launch (gm_gemm_x3_wgrad2: gy is read once per k chunk for both): srcs = [(x, k, sb, period, shift),
    ...] with sb the source's operand scale and the row map of gm_wgrad_src (batch row r reads x row (period ? r
    % period : r) + shift, zero outside x; period / shift 0: plain). The first source's k must be a multiple of
    128 when a second is given. Returns the gradients; None when the shapes do not fit the kernel (the caller
    then runs _wgrad per source)."""
    from . import fused as FU

    Mb, o = gy.shape
    gy = gy.contiguous()
    Ns = [(k + 3) // 4 * 4 for _, k, _, _, _ in srcs]
    ok = (Mb >= 4096 and o % 4 == 0 and gy.data_ptr() % 16 == 0 and len(srcs) in (1, 2)
          and (len(srcs) == 1 or srcs[0][1] % 128 == 0))
    for (x, k, _, _, _), N in zip(srcs, Ns):
        ok = ok and FU.use_x3(k) and N <= x.stride(0) and x.stride(0) % 4 == 0 and x.stride(1) == 1 \
            and x.data_ptr() % 16 == 0
    if not ok:
        return None
    N = sum(Ns)
    tiles = ((o + 127) // 128) * ((N + 127) // 128)
    period = 0
    for _, _, _, per, sh in srcs:
        period = per or period
        if sh:
            period = period or abs(sh)
    kchunk, splits = _wgrad_chunk(Mb, tiles, period)
    if kchunk is None or any((per and per % kchunk) or (sh % kchunk) for _, _, _, per, sh in srcs):
        return None
    lib = FU._setup()
    part = torch.empty(splits, o, N, device=gy.device)
    spec = [L.WgradSrc(x.data_ptr(), x.stride(0), sb.data_ptr(), per, sh, x.shape[0]) for x, _, sb, per, sh in srcs]
    L.check(lib.gm_gemm_x3_wgrad2(gy.data_ptr(), o, C.byref(spec[0]), Ns[0],
                                  C.byref(spec[1]) if len(spec) > 1 else None, Ns[1] if len(spec) > 1 else 0, o, Mb,
                                  kchunk, sa.data_ptr(), part.data_ptr(), N, L.stream_ptr()))
    tot = part.sum(0)
    out, c0 = [], 0
    for (_, k, _, _, _), n in zip(srcs, Ns):
        out.append(tot[:, c0:c0 + k])
        c0 += n
    return out


def _wgrad_pair(gy, x1, k1, x2, k2, sa, sb1, sb2):
    """(gy^T x1[:, :k1], gy^T x2[:, :k2]) in one launch when possible (_wgrad2), else two _wgrad calls."""
    r = _wgrad2(gy, [(x1, k1, sb1, 0, 0), (x2, k2, sb2, 0, 0)], sa)
    return tuple(r) if r is not None else (_wgrad(gy, x1, k1, sa, sb1), _wgrad(gy, x2, k2, sa, sb2))


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act, wcache, tag=None):
        x2, ldx, k = _as_rows(x)
        xs = _amax_slot(x2, ldx, w.shape[0], ctx.needs_input_grad[1])
        zact = act in Z_ACTS and any(ctx.needs_input_grad[:3])
        y = linear_raw(x2, ldx, k, w, b, 0 if zact else act, wcache=wcache, tag=tag, amax=xs)
        keep = y  # the layer output, or for Z_ACTS the pre-activation z (_act_grad)
        if zact:
            y = act_fwd(keep, act)
        ctx.xs = None if xs is None else _finish_scale(xs)
        ctx.act = act
        ctx.wcache = wcache
        ctx.save_for_backward(x2[:, :k] if x2.shape[1] != k else x2, w, keep)
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, w, y = ctx.saved_tensors
        gx, gw, gb = _linear_backward(ctx, gy, x2, w, y, *ctx.needs_input_grad[:3])
        if gx is not None:
            gx = gx.reshape(*ctx.saved_tensors[0].shape[:-1], w.shape[1])
        return gx, gw, gb, None, None, None


def _act_grad(act, gy, y, need_b, want_scale):
    """Backward through the layer activation: (g, bias gradient or None, gradient scale or None).
    y is the layer output, or for Z_ACTS the pre-activation z. relu / elu / tanh / sigmoid / ..: one
    fused pass (gm_act_bwd, derivative from y; gm_act_bwd_z from z). leaky_relu at training sizes: one
    fused pass (gm_leaky_bwd: mask, per-block bias partials, max|g| for the gradient GEMMs' operand scale)."""
    gb = sc = None
    if act > 1:
        # derivative from the output (gm_act_bwd) or the pre-activation (gm_act_bwd_z), any row count
        gy, y = gy.contiguous(), y.contiguous()  # e.g. the slice of a torch.cat's gradient
        rows, cols = gy.shape
        rpb = 64
        g2 = torch.empty_like(gy)
        part = torch.empty((rows + rpb - 1) // rpb, cols, device=gy.device)
        sc = torch.empty(1, device=gy.device) if want_scale and rows >= 4096 else None
        fn = L.lib().gm_act_bwd_z if act in Z_ACTS else L.lib().gm_act_bwd
        L.check(fn(gy.data_ptr(), y.data_ptr(), rows, cols, act, g2.data_ptr(), part.data_ptr(), rpb, L.ptr(sc), _s()))
        gy = g2
        if need_b:
            gb = part.sum(0)
    elif act == 1:
        if gy.is_contiguous() and y.is_contiguous() and gy.shape[0] >= 4096:
            rows, cols = gy.shape
            rpb = 64
            g2 = torch.empty_like(gy)
            part = torch.empty((rows + rpb - 1) // rpb, cols, device=gy.device)
            sc = torch.empty(1, device=gy.device)
            L.check(L.lib().gm_leaky_bwd(gy.data_ptr(), y.data_ptr(), rows, cols, 0.01, g2.data_ptr(),
                                         part.data_ptr(), rpb, sc.data_ptr(), _s()))
            gy = g2
            if need_b:
                gb = part.sum(0)
        else:
            gy = torch.where(y >= 0, gy, 0.01 * gy)
    if sc is None and want_scale and gy.is_contiguous() and gy.shape[0] >= 4096:
        sc = _gy_scale(gy)  # one scale for both gradient GEMMs
    if gb is None and need_b:
        gb = _colsum(gy)
    return gy, gb, sc


def _colsum(g):
    """Column sums of a [rows, cols] gradient (a bias gradient). Above 64 k rows in two stages:
    256-row partials first (one torch reduction of millions of rows to ~100 columns ran at ~0.15 TB/s,
    e.g. the SL head over 6.5 M rows)."""
    rows = g.shape[0]
    if rows < 65536 or not g.is_contiguous():
        return g.sum(0)
    r0 = rows // 256 * 256
    s = g[:r0].view(r0 // 256, 256, -1).sum(1).sum(0)
    return s + g[r0:].sum(0) if r0 < rows else s


def _linear_backward(ctx, gy, x2, w, y, need_x, need_w, need_b):
    """Gradients of y = act(x2 @ w^T + b) (ctx.act, ctx.wcache, ctx.xs = published max|x| scale
    or None): the activation backward, then the split-f16 input- and weight-gradient GEMMs
    sharing one gradient scale."""
    gy, gb, sc = _act_grad(ctx.act, gy.reshape(-1, w.shape[0]), y, need_b, need_x and need_w)
    gx = _dgrad(gy, w, ctx.wcache, sc) if need_x else None
    gw = _wgrad(gy, x2, w.shape[1], sc, ctx.xs) if need_w else None
    return gx, gw, gb


class _JointLinearFn(torch.autograd.Function):
    """First DQN layer on the joint observation [env obs | NetMon graph obs] (src/model.py:187-203
    with src/env/wrapper.py:106-109) without materialising it: one split-f16 GEMM over two dense
    A sources [graph | env] (weights column-reordered once, fused.pack_dqn_first) that publishes
    max|A| for the weight gradient; backward computes the input gradient of the graph part only
    (the env observation is data) and the weight gradient per source."""

    @staticmethod
    def forward(ctx, graph, env_obs, w, b, lin):
        from . import fused as FU

        R, G = graph.shape
        od = env_obs.shape[1]
        wp, ldw, bp, x3 = FU.pack_dqn_first(lin, od)
        xs = torch.zeros(1, device=graph.device) if ctx.needs_input_grad[2] else None
        y = torch.empty(R, w.shape[0], device=graph.device)
        zact = lin.act in Z_ACTS
        FU.gemm(FU.dense(graph.data_ptr(), G, G, amax=None if xs is None else xs.data_ptr()),
                FU.dense(env_obs.data_ptr(), env_obs.stride(0), od), wp.data_ptr(), ldw, bp.data_ptr(), R, w.shape[0],
                epi_code(0 if zact else lin.act), y.data_ptr(), w.shape[0],
                tag=lin.tag and f"linear:{lin.tag}:{R}x{w.shape[0]}x{G}+{od}", x3=x3)
        ctx.xs = None if xs is None else _finish_scale(xs)
        ctx.act = lin.act
        if not hasattr(lin, "_wc_graph"):
            lin._wc_graph = _WeightCache()
        ctx.wcache_graph = lin._wc_graph
        ctx.save_for_backward(graph, env_obs, w, y)  # Z_ACTS: y holds z (_act_grad)
        return act_fwd(y, lin.act) if zact else y

    @staticmethod
    def backward(ctx, gy):
        graph, env_obs, w, y = ctx.saved_tensors
        od = env_obs.shape[1]
        n = ctx.needs_input_grad
        g, gb, sc = _act_grad(ctx.act, gy, y, n[3], n[0] and n[2])
        gg = _dgrad(g, w[:, od:], ctx.wcache_graph, sc) if n[0] else None
        gw = None
        if n[2]:
            gw = torch.cat([_wgrad(g, env_obs, od, sc, ctx.xs), _wgrad(g, graph, graph.shape[1], sc, ctx.xs)], 1)
        return gg, None, gw, gb, None


def joint_first_layer_ok(graph2d, env2d):
    """The two-source first layer needs the split-f16 form, training batch sizes and 16-byte rows."""
    from . import fused as FU

    return (FU.use_x3(512) and graph2d.shape[0] >= 4096 and graph2d.is_contiguous() and graph2d.shape[1] % 32 == 0
            and env2d.stride(1) == 1 and env2d.stride(0) % 4 == 0 and env2d.data_ptr() % 16 == 0
            and graph2d.data_ptr() % 16 == 0)


class _RoutingEncFn(torch.autograd.Function):
    """First NetMon encoder layer on routing node observations with gradient: forward on the
    12-column gather (gm_routing_node_encoder, exact fp32), backward as a Linear (the node
    observations are data: no input gradient)."""

    @staticmethod
    def forward(ctx, x, w, b, nbr, lin, G, N):
        from . import fused as FU

        y = torch.empty(x.shape[0], w.shape[0], device=x.device)
        zact = lin.act in Z_ACTS
        FU.routing_encoder(lin, x, nbr, G, N, y, act=0 if zact else None)
        ctx.act, ctx.wcache, ctx.xs = lin.act, lin._wc, None
        ctx.save_for_backward(x, w, y)  # Z_ACTS: y holds z (_act_grad)
        return act_fwd(y, lin.act) if zact else y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        _, gw, gb = _linear_backward(ctx, gy, x, w, y, False, ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        return None, gw, gb, None, None, None, None


class Linear(nn.Linear):
    """nn.Linear whose forward runs the fused MFMA kernel (act: GM_ACT_* code, 0 none, 1 leaky_relu)."""

    def __init__(self, in_features, out_features, bias=True, act=0):
        super().__init__(in_features, out_features, bias)
        self.act = act
        self._wc = _WeightCache()
        self.tag = None

    def forward(self, x):
        if x.shape[-1] != self.in_features:
            raise ValueError(f"Linear expects {self.in_features} features, got {x.shape[-1]}")
        lead = x.shape[:-1]
        y = LinearFn.apply(x.reshape(-1, x.shape[-1]), self.weight, self.bias, self.act, self._wc, self.tag)
        return y.reshape(*lead, self.out_features)


class MLP(nn.Module):
    """src/model.py:13-42 (the activation after every layer, including the output by default;
    activation: a torch.nn.functional name of ACTIVATIONS, the reference's activation_fn)."""

    def __init__(self, in_features, mlp_units, activation_on_output=True, activation="leaky_relu"):
        super().__init__()
        if isinstance(mlp_units, int):
            mlp_units = [mlp_units]
        act = act_code(activation)
        self.linear_layers = nn.ModuleList()
        prev = in_features
        for i, u in enumerate(mlp_units):
            last = i == len(mlp_units) - 1
            self.linear_layers.append(Linear(prev, u, act=0 if (last and not activation_on_output) else act))
            prev = u
        self.out_features = prev

    def forward(self, x):
        for lin in self.linear_layers:
            x = lin(x)
        return x

    def forward_into(self, x2d, ldx, k, scratch, n_layers=None):
        """no-grad fast path over a strided row buffer (e.g. the joint observation); the first
        n_layers layers (default all)."""
        h, ld, kk = x2d, ldx, k
        for i, lin in enumerate(self.linear_layers[:n_layers]):
            out = scratch(i, x2d.shape[0], lin.out_features)
            linear_raw(h, ld, kk, lin.weight, lin.bias, lin.act, out=out, ldy=out.stride(0), wcache=lin._wc,
                       tag=lin.tag)
            h, ld, kk = out, out.stride(0), lin.out_features
        return h


class _Aggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, nbr, mode):
        G, N, deg = nbr.shape
        H = h.shape[-1]
        out = torch.empty_like(h)
        with L.timed(f"mp_aggregate:{G * N}x{H}"):
            L.check(L.lib().gm_mp_aggregate(L.ptr(h), L.ptr(nbr), G, N, deg, H, mode, L.ptr(out), _s()))
        ctx.save_for_backward(nbr)
        ctx.mode = mode
        return out

    @staticmethod
    def backward(ctx, g):
        (nbr,) = ctx.saved_tensors
        G, N, deg = nbr.shape
        g = g.contiguous()
        dh = torch.empty_like(g)
        L.check(L.lib().gm_mp_aggregate_bwd(L.ptr(g), L.ptr(nbr), G, N, deg, g.shape[-1], ctx.mode, L.ptr(dh), _s()))
        return dh, None, None


def mp_aggregate(h, nbr, mode=SUM):
    """SimpleAggregation (src/model.py:206-229): rows of h [G*N, H] summed over {n} ∪ nbr(n)."""
    return _Aggregate.apply(h.contiguous(), nbr, mode)


class _Readout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hf, hp, nbr, agent_node, out, col0):
        G, N, deg = nbr.shape
        H = hf.shape[-1]
        R = N if agent_node is None else agent_node.shape[1]
        if out is None:
            res = torch.empty(G * R, (deg + 1) * H, device=hf.device)
            dst, stride = res, res.stride(0)
        else:
            res = None
            dst = out.view(-1, out.shape[-1])[:, col0:]
            stride = out.shape[-1]
        with L.timed(f"netmon_readout:{G * R}x{(deg + 1) * H}"):
            L.check(L.lib().gm_netmon_readout(L.ptr(hf), L.ptr(hp), L.ptr(nbr), L.ptr(agent_node), G, N, R, deg, H,
                                              L.ptr(dst), stride, _s()))
        ctx.save_for_backward(nbr, agent_node if agent_node is not None else torch.empty(0))
        ctx.has_map = agent_node is not None
        ctx.H = H
        return res if res is not None else out

    @staticmethod
    def backward(ctx, g):
        nbr, an = ctx.saved_tensors
        an = an if ctx.has_map else None
        G, N, deg = nbr.shape
        R = N if an is None else an.shape[1]
        g = g.contiguous()
        dhf = torch.empty(G * N, ctx.H, device=g.device)
        dhp = torch.empty(G * N, ctx.H, device=g.device)
        L.check(L.lib().gm_netmon_readout_bwd(L.ptr(g), g.shape[-1], L.ptr(nbr), L.ptr(an), G, N, R, deg, ctx.H,
                                              L.ptr(dhf), L.ptr(dhp), _s()))
        return dhf, dhp, None, None, None, None


def netmon_readout(h_final, h_prev, nbr, agent_node=None, out=None, col0=0):
    """NetMon readout (src/model.py:457-474, 582-631): rows [h(v), h_prev(nbr(v, 0..2))]
    for v = agent_node[g, r] (output_to_network_obs) or every node. With `out` the rows
    are written into columns [col0, col0 + 4H) of an existing buffer (no-grad path)."""
    return _Readout.apply(h_final.contiguous(), h_prev.contiguous(), nbr, agent_node, out, col0)


class _LSTMPointwise(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gates, c):
        M, H4 = gates.shape
        H = H4 // 4
        h1 = torch.empty(M, H, device=gates.device)
        c1 = torch.empty(M, H, device=gates.device)
        need = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        act = torch.empty_like(gates) if need else None
        with L.timed(f"lstm_pointwise:{M}x{H}"):
            L.check(L.lib().gm_lstm_pointwise(L.ptr(gates), L.ptr(c), M, H, L.ptr(h1), L.ptr(c1), L.ptr(act), _s()))
        if need:
            ctx.save_for_backward(act, c, c1)
        return h1, c1

    @staticmethod
    def backward(ctx, dh1, dc1):
        act, c, c1 = ctx.saved_tensors
        M, H = c.shape
        dg = torch.empty(M, 4 * H, device=c.device)
        dc = torch.empty(M, H, device=c.device)
        dh1 = None if dh1 is None else dh1.contiguous()
        dc1 = None if dc1 is None else dc1.contiguous()
        L.check(L.lib().gm_lstm_pointwise_bwd(L.ptr(dh1), L.ptr(dc1), L.ptr(act), L.ptr(c), L.ptr(c1), M, H,
                                              L.ptr(dg), L.ptr(dc), None, _s()))
        return dg, dc


class _LSTMCellFn(torch.autograd.Function):
    """One LSTMCell step as one autograd node: gates = [x|h] W^T + b (split-f16 GEMM that
    publishes max|[x|h]| for the weight gradient) and the gate math; backward runs the gate-math
    backward (publishing max|dgates|) straight into the two gradient GEMMs, so neither operand
    scale costs a pass of its own."""

    @staticmethod
    def forward(ctx, xh, w, b, c, wcache, tag, packed=None):
        x2, ldx, k = _as_rows(xh)
        xs = _amax_slot(x2, ldx, w.shape[0], ctx.needs_input_grad[1])
        M, H4 = x2.shape[0], w.shape[0]
        H = H4 // 4
        h1 = torch.empty(M, H, device=x2.device)
        c1 = torch.empty(M, H, device=x2.device)
        act = torch.empty(M, H4, device=x2.device)
        if packed is not None:
            # gate math in the GEMM epilogue (interleaved gate tiles, fused.pack_lstm): h', c' and
            # the gate activations for backward straight from the accumulators, no gates tensor
            from . import fused as FU

            wp, ldw, bp, x3 = packed
            FU.gemm(FU.dense(x2.data_ptr(), ldx, k, amax=None if xs is None else xs.data_ptr()), None, wp.data_ptr(),
                    ldw, bp.data_ptr(), M, H4, FU.GM_EPI_LSTM, h1.data_ptr(), H, c1.data_ptr(), H, c.data_ptr(), H,
                    act.data_ptr(), tag=tag and f"lstm:{tag}:{M}x{H4}x{k}", x3=x3)
        else:
            gates = linear_raw(x2, ldx, k, w, b, 0, wcache=wcache, tag=tag, amax=xs)
            L.check(L.lib().gm_lstm_pointwise(L.ptr(gates), L.ptr(c), M, H, L.ptr(h1), L.ptr(c1), L.ptr(act), _s()))
        ctx.xs = None if xs is None else _finish_scale(xs)
        ctx.wcache = wcache
        ctx.save_for_backward(x2[:, :k] if x2.shape[1] != k else x2, w, act, c, c1)
        return h1, c1

    @staticmethod
    def backward(ctx, dh1, dc1):
        x2, w, act, c, c1 = ctx.saved_tensors
        M, H = c.shape
        dg = torch.empty(M, 4 * H, device=c.device)
        dc = torch.empty(M, H, device=c.device)
        sc = torch.empty(1, device=c.device)
        dh1 = None if dh1 is None else dh1.contiguous()
        dc1 = None if dc1 is None else dc1.contiguous()
        L.check(L.lib().gm_lstm_pointwise_bwd(L.ptr(dh1), L.ptr(dc1), L.ptr(act), L.ptr(c), L.ptr(c1), M, H,
                                              L.ptr(dg), L.ptr(dc), L.ptr(sc), _s()))
        n = ctx.needs_input_grad
        gx = _dgrad(dg, w, ctx.wcache, sc) if n[0] else None
        gw = _wgrad(dg, x2, w.shape[1], sc, ctx.xs) if n[1] else None
        gb = dg.sum(0) if n[2] else None
        return gx, gw, gb, dc if n[3] else None, None, None, None


class _LSTMCell2Fn(torch.autograd.Function):
    """_LSTMCellFn with x and h as the GEMM's two dense A sources (no [x | h] tensor in the forward,
    no slicing of its gradient in the backward): gates in the epilogue (fused.pack_lstm), max |[x | h]|
    published for the weight gradient; backward = the gate-math backward, ONE input-gradient GEMM whose
    split output writes dx and dh apart (gm_gemm_x3_dgrad), and the weight gradients of W_ih / W_hh."""

    @staticmethod
    def forward(ctx, x, h, w_ih, w_hh, b_ih, b_hh, c, cell):
        from . import fused as FU

        M, I = x.shape
        H = h.shape[1]
        wp, ldw, bp, x3 = FU.pack_lstm(cell)
        need_w = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        xs = torch.zeros(1, device=x.device) if need_w else None
        h1 = torch.empty(M, H, device=x.device)
        c1 = torch.empty(M, H, device=x.device)
        act = torch.empty(M, 4 * H, device=x.device)
        tag = cell.tag and f"lstm:{cell.tag}:{M}x{4 * H}x{I + H}"
        FU.gemm(FU.dense(x.data_ptr(), x.stride(0), I, amax=None if xs is None else xs.data_ptr()),
                FU.dense(h.data_ptr(), h.stride(0), H), wp.data_ptr(), ldw, bp.data_ptr(), M, 4 * H, FU.GM_EPI_LSTM,
                h1.data_ptr(), H, c1.data_ptr(), H, c.data_ptr(), c.stride(0), act.data_ptr(), tag=tag, x3=x3)
        ctx.xs = None if xs is None else _finish_scale(xs)
        ctx.cell = cell
        ctx.save_for_backward(x, h, w_ih, w_hh, act, c, c1)
        return h1, c1

    @staticmethod
    def backward(ctx, dh1, dc1):
        import ctypes as C

        from . import fused as FU

        x, h, w_ih, w_hh, act, c, c1 = ctx.saved_tensors
        M, H = c.shape
        I = x.shape[1]
        dg = torch.empty(M, 4 * H, device=c.device)
        dc = torch.empty(M, H, device=c.device)
        sc = torch.empty(1, device=c.device)
        dh1 = None if dh1 is None else dh1.contiguous()
        dc1 = None if dc1 is None else dc1.contiguous()
        cc = c.contiguous()
        L.check(L.lib().gm_lstm_pointwise_bwd(L.ptr(dh1), L.ptr(dc1), L.ptr(act), L.ptr(cc), L.ptr(c1), M, H,
                                              L.ptr(dg), L.ptr(dc), L.ptr(sc), _s()))
        n = ctx.needs_input_grad
        dx = dh = None
        if n[0] or n[1]:
            from . import train_seq as TS

            # [W_ih | W_hh]^T packed once per parameter version on the cell (train_seq's cache)
            x3 = TS._lstm_x3t(ctx.cell)
            dx = torch.empty(M, I, device=c.device)
            dh = torch.empty(M, H, device=c.device)
            a = FU.dense(dg.data_ptr(), 4 * H, 4 * H, scale=sc.data_ptr())
            L.check(FU._setup().gm_gemm_x3_dgrad(C.byref(a), x3.wp.data_ptr(), x3.sinv.data_ptr(), M, I + H, I, None,
                                                 0, dx.data_ptr(), I, dh.data_ptr(), H, None, None, _s()))
        gwi = _wgrad(dg, x, I, sc, ctx.xs) if n[2] else None
        gwh = _wgrad(dg, h, H, sc, ctx.xs) if n[3] else None
        gb = dg.sum(0) if (n[4] or n[5]) else None
        return (dx if n[0] else None, dh if n[1] else None, gwi, gwh, gb if n[4] else None,
                (gb.clone() if n[4] else gb) if n[5] else None, dc if n[6] else None, None)


def _two_source_ok(x, h):
    return (x.dim() == 2 and h.dim() == 2 and x.stride(1) == 1 and h.stride(1) == 1 and x.stride(0) % 4 == 0
            and h.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0 and h.data_ptr() % 16 == 0 and x.shape[1] % 32 == 0)


class LSTMCell(nn.Module):
    """nn.LSTMCell parameters/semantics; gates = [x|h] @ [W_ih|W_hh]^T + (b_ih + b_hh)
    in one MFMA GEMM, gate math in gm_lstm_pointwise."""

    def __init__(self, input_size, hidden_size):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.weight_ih = nn.Parameter(torch.empty(4 * hidden_size, input_size))
        self.weight_hh = nn.Parameter(torch.empty(4 * hidden_size, hidden_size))
        self.bias_ih = nn.Parameter(torch.empty(4 * hidden_size))
        self.bias_hh = nn.Parameter(torch.empty(4 * hidden_size))
        stdv = 1.0 / math.sqrt(hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -stdv, stdv)
        self._wc = _WeightCache()
        self.tag = None

    def forward(self, x, state):
        h, c = state
        if (torch.is_grad_enabled() and x.shape[0] >= 4096 and self.hidden_size % 32 == 0
                and self.input_size == self.hidden_size and _x3_rows_ok(x, x.stride(0), 4 * self.hidden_size)
                and _two_source_ok(x, h) and c.is_contiguous()
                and (self.weight_ih.requires_grad or x.requires_grad or h.requires_grad)):
            return _LSTMCell2Fn.apply(x, h, self.weight_ih, self.weight_hh, self.bias_ih, self.bias_hh, c, self)
        xh = torch.cat([x, h], -1)
        w = torch.cat([self.weight_ih, self.weight_hh], 1)
        b = self.bias_ih + self.bias_hh
        if torch.is_grad_enabled() and (w.requires_grad or xh.requires_grad):
            if xh.shape[0] >= 4096 and _x3_rows_ok(xh, xh.stride(0), w.shape[0]):
                from . import fused as FU

                packed = FU.pack_lstm(self) if self.hidden_size % 32 == 0 else None
                return _LSTMCellFn.apply(xh, w, b, c.contiguous(), None, self.tag, packed)
            gates = LinearFn.apply(xh, w, b, 0, None, self.tag)
        else:
            gates = linear_raw(xh, xh.stride(0), xh.shape[1], w, b, 0, tag=self.tag)
        return _LSTMPointwise.apply(gates, c.contiguous())


class _LNLSTMFn(torch.autograd.Function):
    """LayerNorm-LSTM gate math after the two gate GEMMs (src/layernormlstm.py:24-42) as one
    autograd node on the HIP kernels: gm_lnlstm_fwd (one wave per row, the three LayerNorms as
    wave reductions, row statistics saved) and gm_lnlstm_bwd (the hand-differentiated cell:
    gradients of both raw gate rows and of c, per-wave partials of the LayerNorm and bias
    gradients). The raw gate rows are the GEMMs' own outputs, so no activation tensor is saved."""

    @staticmethod
    def forward(ctx, gi, gh, c, wi, bi, wh, bh, bias, wc, bc, eps):
        M, H4 = gi.shape
        H = H4 // 4
        h1 = torch.empty(M, H, device=gi.device)
        c1 = torch.empty(M, H, device=gi.device)
        stats = torch.empty(M, 8, device=gi.device)
        L.check(L.lib().gm_lnlstm_fwd(gi.data_ptr(), gi.stride(0), gh.data_ptr(), gh.stride(0), c.data_ptr(),
                                      c.stride(0), wi.data_ptr(), bi.data_ptr(), wh.data_ptr(), bh.data_ptr(),
                                      bias.data_ptr(), wc.data_ptr(), bc.data_ptr(), M, H, eps, h1.data_ptr(), H,
                                      c1.data_ptr(), H, stats.data_ptr(), _s()))
        ctx.save_for_backward(gi, gh, c, wi, bi, wh, bh, bias, wc, bc, stats)
        ctx.eps = eps
        return h1, c1

    @staticmethod
    def backward(ctx, dh1, dc1):
        gi, gh, c, wi, bi, wh, bh, bias, wc, bc, stats = ctx.saved_tensors
        M, H4 = gi.shape
        H = H4 // 4
        dh1 = None if dh1 is None else dh1.contiguous()
        dc1 = None if dc1 is None else dc1.contiguous()
        dgi = torch.empty(M, H4, device=gi.device)
        dgh = torch.empty(M, H4, device=gi.device)
        dc = torch.empty(M, H, device=gi.device)
        rpw = 8
        part = torch.empty((M + rpw - 1) // rpw, 14 * H, device=gi.device)
        L.check(L.lib().gm_lnlstm_bwd(gi.data_ptr(), gi.stride(0), gh.data_ptr(), gh.stride(0), c.data_ptr(),
                                      c.stride(0), wi.data_ptr(), bi.data_ptr(), wh.data_ptr(), bh.data_ptr(),
                                      bias.data_ptr(), wc.data_ptr(), bc.data_ptr(), stats.data_ptr(),
                                      L.ptr(dh1), H, L.ptr(dc1), H, M, H, rpw, dgi.data_ptr(), H4, dgh.data_ptr(), H4,
                                      dc.data_ptr(), H, part.data_ptr(), _s()))
        ps = part.sum(0)
        dwi, dwh, db, dwc, dbc = ps[:H4], ps[H4:2 * H4], ps[2 * H4:3 * H4], ps[3 * H4:3 * H4 + H], ps[3 * H4 + H:]
        # d ln_in_b = d ln_hid_b = d bias_ih: separate tensors (each may become a .grad modified in place)
        return dgi, dgh, dc, dwi, db, dwh, db.clone(), db.clone(), dwc, dbc, None


class LayerNormLSTMCell(nn.Module):
    """src/layernormlstm.py:8-42 (LN on the input and hidden gate pre-activations and on
    the cell, single bias): the two gate GEMMs on the MFMA kernel (LinearFn: split-f16 forward,
    input and weight gradients), the LayerNorms and gate math in gm_lnlstm_fwd / gm_lnlstm_bwd."""

    def __init__(self, input_size, hidden_size):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.weight_ih = nn.Parameter(torch.empty(4 * hidden_size, input_size))
        self.weight_hh = nn.Parameter(torch.empty(4 * hidden_size, hidden_size))
        self.bias_ih = nn.Parameter(torch.empty(4 * hidden_size))
        stdv = 1.0 / math.sqrt(hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -stdv, stdv)
        self.ln_input = nn.LayerNorm(4 * hidden_size)
        self.ln_hidden = nn.LayerNorm(4 * hidden_size)
        self.ln_cell = nn.LayerNorm(hidden_size)
        self._wci, self._wch = _WeightCache(), _WeightCache()
        self.tag = None

    def forward(self, x, state):
        hx, cx = state
        gi = LinearFn.apply(x, self.weight_ih, None, 0, self._wci, self.tag)
        gh = LinearFn.apply(hx, self.weight_hh, None, 0, self._wch, self.tag and self.tag + ".hh")
        li, lh, lc = self.ln_input, self.ln_hidden, self.ln_cell
        return _LNLSTMFn.apply(gi.reshape(-1, 4 * self.hidden_size), gh.reshape(-1, 4 * self.hidden_size),
                               cx.contiguous(), li.weight, li.bias, lh.weight, lh.bias, self.bias_ih, lc.weight,
                               lc.bias, float(li.eps))


class _GRUFn(torch.autograd.Function):
    """nn.GRUCell gate math after the two gate GEMMs as one autograd node (gm_gru_pointwise /
    gm_gru_bwd; backward recomputes r, z, n from the saved gate rows)."""

    @staticmethod
    def forward(ctx, gi, gh, h):
        M, H3 = gi.shape
        H = H3 // 3
        h1 = torch.empty(M, H, device=gi.device)
        L.check(L.lib().gm_gru_pointwise(gi.data_ptr(), gi.stride(0), gh.data_ptr(), gh.stride(0), h.data_ptr(),
                                         h.stride(0), M, H, h1.data_ptr(), H, _s()))
        ctx.save_for_backward(gi, gh, h)
        return h1

    @staticmethod
    def backward(ctx, dh1):
        gi, gh, h = ctx.saved_tensors
        M, H3 = gi.shape
        H = H3 // 3
        dh1 = dh1.contiguous()
        dgi = torch.empty(M, H3, device=gi.device)
        dgh = torch.empty(M, H3, device=gi.device)
        dh = torch.empty(M, H, device=gi.device)
        L.check(L.lib().gm_gru_bwd(gi.data_ptr(), gi.stride(0), gh.data_ptr(), gh.stride(0), h.data_ptr(), h.stride(0),
                                   dh1.data_ptr(), H, M, H, dgi.data_ptr(), H3, dgh.data_ptr(), H3, dh.data_ptr(), H,
                                   _s()))
        return dgi, dgh, dh


class GRUCell(nn.Module):
    """nn.GRUCell semantics (r, z, n): the two gate GEMMs on the MFMA kernel (LinearFn), the gate
    math in gm_gru_pointwise / gm_gru_bwd."""

    def __init__(self, input_size, hidden_size):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.weight_ih = nn.Parameter(torch.empty(3 * hidden_size, input_size))
        self.weight_hh = nn.Parameter(torch.empty(3 * hidden_size, hidden_size))
        self.bias_ih = nn.Parameter(torch.empty(3 * hidden_size))
        self.bias_hh = nn.Parameter(torch.empty(3 * hidden_size))
        stdv = 1.0 / math.sqrt(hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -stdv, stdv)
        self._wci, self._wch = _WeightCache(), _WeightCache()
        self.tag = None

    def forward(self, x, h):
        gi = LinearFn.apply(x, self.weight_ih, self.bias_ih, 0, self._wci, self.tag)
        gh = LinearFn.apply(h, self.weight_hh, self.bias_hh, 0, self._wch, self.tag and self.tag + ".hh")
        H = self.hidden_size
        return _GRUFn.apply(gi.reshape(-1, 3 * H), gh.reshape(-1, 3 * H), h.contiguous())


def dense_to_nbr(mask, max_degree=None):
    """(I + A) float mask [B, N, N] -> neighbour table int32 [B, N, deg] (ascending, -1 pad).
    deg = max_degree when given (the reference's NetMon.forward argument, src/model.py:451-474;
    no host sync), else the largest degree in the batch (one device -> host read)."""
    B, N, _ = mask.shape
    m = (mask != 0) & ~torch.eye(N, dtype=torch.bool, device=mask.device)
    if max_degree is not None:
        deg = int(max_degree)
    else:
        deg = int(m.sum(-1).max().item()) if m.numel() else 0
    deg = min(max(deg, 1), N)
    ids = torch.arange(N, device=mask.device).expand(B, N, N)
    key = torch.where(m, ids, ids + N)
    srt = key.sort(-1).values[..., :deg]
    return torch.where(srt < N, srt, torch.full_like(srt, -1)).to(torch.int32).contiguous()


def node_agent_to_index(node_agent):
    """node-agent matrix [B, N, A] -> node index of every agent int32 [B, A]."""
    return node_agent.argmax(1).to(torch.int32).contiguous()


class NetMon(nn.Module):
    """src/model.py:256-650 for agg_type sum|mean, rnn lstm|lnlstm|gru, carry-over state.

    forward(x, mask, node_agent_matrix, max_degree=None, no_agent_mapping=False) keeps the
    reference signature (dense (I+A) mask / node-agent matrix); forward_graph() is the
    native entry point taking the neighbour table nbr [B, N, 3] and agent_node [B, A].
    """

    def __init__(self, in_features, hidden_features, encoder_units, iterations, rnn_type="lstm",
                 rnn_carryover=True, agg_type="sum", output_neighbor_hidden=True, output_global_hidden=False,
                 activation="leaky_relu"):
        super().__init__()
        if agg_type not in ("sum", "mean"):
            raise NotImplementedError(f"agg_type {agg_type!r}: only sum/mean are built (torch_geometric variants "
                                      "are out of scope)")
        if not rnn_carryover and iterations < 1:
            raise ValueError("rnn_carryover=False needs netmon iterations >= 1 (the reference's update "
                             "cell output is the stored state)")
        self.encode = MLP(in_features, (*encoder_units, hidden_features), activation=activation)
        self._hc = None  # carry-over LSTM state kept as its (h, c) rows (training), see state
        self.state = None
        self.iterations = iterations
        self.output_neighbor_hidden = output_neighbor_hidden
        self.output_global_hidden = output_global_hidden
        self.rnn_carryover = rnn_carryover
        self.agg_type_str = agg_type
        self.agg_mode = SUM if agg_type == "sum" else MEAN
        self.rnn_type = rnn_type
        if rnn_type == "lstm":
            self.rnn_obs = LSTMCell(hidden_features, hidden_features)
            self.rnn_update = LSTMCell(hidden_features, hidden_features)
            self.num_states = 2
        elif rnn_type == "lnlstm":
            self.rnn_obs = LayerNormLSTMCell(hidden_features, hidden_features)
            self.rnn_update = LayerNormLSTMCell(hidden_features, hidden_features)
            self.num_states = 2
        elif rnn_type == "gru":
            self.rnn_obs = GRUCell(hidden_features, hidden_features)
            self.rnn_update = GRUCell(hidden_features, hidden_features)
            self.num_states = 1
        else:
            raise NotImplementedError(f"rnn_type {rnn_type!r}")
        # without carry-over the state also keeps the update cell's output (src/model.py:380-391)
        self.cell_states = self.num_states
        if not rnn_carryover:
            self.num_states *= 2
        self.hidden_features = hidden_features
        self.state_size = hidden_features * self.num_states

    # The reference's mutable state tensor [B, N, state_size] (src/model.py:403-415, 447-449). A
    # carry-over lstm / lnlstm step with gradient leaves it as its (h, c) row tensors instead
    # (no stack, no split copies on the next step); reading .state stacks them on demand.
    @property
    def state(self):
        if self._state is None and self._hc is not None:
            h, c, B, N = self._hc
            self._state = torch.stack((h, c), 1).reshape(B, N, self.state_size)
        return self._state

    @state.setter
    def state(self, value):
        self._state = value
        self._hc = None

    def state_hc(self):
        """(h, c, B, N) of a state held as rows, or None."""
        return self._hc

    def set_state_hc(self, h, c, B, N):
        self._state = None
        self._hc = (h, c, B, N)

    def save_state(self):
        return self._state, self._hc

    def restore_state(self, tok):
        self._state, self._hc = tok

    def get_out_features(self):
        """src/model.py:403-415 for routing graphs (max degree 3): h, [global mean], [3 neighbours]."""
        return self.hidden_features * (1 + (1 if self.output_global_hidden else 0) +
                                       (3 if self.output_neighbor_hidden else 0))

    def get_state_size(self):
        return self.state_size

    def _encode(self, x2, nbr, B, N):
        """Encoder MLP; with gradient at training batch sizes the first layer runs on the routing
        node-observation gather (_RoutingEncFn) instead of the dense K = 4N+8 GEMM."""
        from . import fused as FU

        layers = self.encode.linear_layers
        if torch.is_grad_enabled() and x2.shape[0] >= 4096 and not x2.requires_grad and \
                FU.routing_encoder_ok(layers[0], N, x2.shape[1], nbr):
            lin = layers[0]
            h = _RoutingEncFn.apply(x2.contiguous(), lin.weight, lin.bias, nbr.contiguous(), lin, B, N)
            for lin in layers[1:]:
                h = lin(h)
            return h
        return self.encode(x2)

    def _cell(self, cell, x, h, c):
        if self.rnn_type == "gru":
            return cell(x, h), None
        return cell(x, (h, c))

    def encode_nodes(self, x, nbr):
        """The encoder MLP over every node row ([B*N, H]): forward_graph's first stage, for callers
        that unroll NetMon several times on the same observations (sl.py) and pass it as `enc`."""
        B, N, Fdim = x.shape
        return self._encode(x.reshape(B * N, Fdim), nbr, B, N)

    def forward_graph(self, x, nbr, agent_node=None, out=None, out_col=0, enc=None):
        """x [B, N, F] node observations, nbr int32 [B, N, deg], agent_node int32 [B, A] or None;
        enc: encode_nodes(x, nbr) computed once by the caller (the same values the encoder gives).
        Returns [B, A or N, 4H] (or writes into `out` [B, A, W] at column out_col)."""
        B, N, Fdim = x.shape
        H = self.hidden_features
        nc = self.cell_states
        if self._hc is not None:
            hs, cs = self._hc[0], self._hc[1]
            st = None
        else:
            if self.state is None:
                self.state = torch.zeros(B, N, self.state_size, device=x.device)
            st = self.state.reshape(B * N, self.num_states, H)
            hs, cs = st[:, 0].contiguous(), (st[:, 1].contiguous() if nc == 2 else None)
        h = enc if enc is not None else self._encode(x.reshape(B * N, Fdim), nbr, B, N)
        h, c = self._cell(self.rnn_obs, h, hs, cs)
        h0, c0 = h, c
        last_nbr = torch.zeros_like(h) if self.iterations <= 0 else None
        for it in range(self.iterations):
            if it == self.iterations - 1:
                last_nbr = h
            M = mp_aggregate(h, nbr, self.agg_mode)
            hin, cin = h, c
            if not self.rnn_carryover and it == 0:  # src/model.py:538-549
                hin = st[:, nc].contiguous()
                cin = st[:, nc + 1].contiguous() if nc == 2 else None
            h, c = self._cell(self.rnn_update, M, hin, cin)
        if self.rnn_carryover and c is not None and torch.is_grad_enabled():
            self.set_state_hc(h, c, B, N)  # stacked only when .state is read
        elif self.rnn_carryover:
            self.state = (torch.stack((h, c), 1) if c is not None else h.unsqueeze(1)).reshape(B, N, self.state_size)
        elif nc == 2:
            self.state = torch.stack((h0, c0, h, c), 1).reshape(B, N, self.state_size)
        else:
            # the reference stacks (h0[None], h1[None]) and its transpose(0, 1) + reshape keeps
            # the component-major order: rows hold [h0 of all nodes | h1 of all nodes]
            # (src/model.py:566-567, 447-449)
            self.state = torch.cat((h0.reshape(-1), h.reshape(-1))).reshape(B, N, self.state_size)
        if self.output_global_hidden:
            # [h | mean over the graph's nodes of h | neighbour h] (src/model.py:458-469, 624-627)
            hv = h.reshape(B, N, H)
            parts = [hv, hv.mean(dim=1, keepdim=True).expand(B, N, H)]
            if self.output_neighbor_hidden:
                parts.append(netmon_readout(h, last_nbr, nbr, None).reshape(B, N, -1)[..., H:])
            full = torch.cat(parts, -1)
            if agent_node is not None:
                full = torch.gather(full, 1, agent_node.long().unsqueeze(-1).expand(-1, -1, full.shape[-1]))
            if out is not None:
                out[..., out_col:out_col + full.shape[-1]] = full
                return out
            return full
        if not self.output_neighbor_hidden:
            hv = h.reshape(B, N, H)
            if agent_node is None:
                return hv
            return torch.gather(hv, 1, agent_node.long().unsqueeze(-1).expand(-1, -1, H))
        res = netmon_readout(h, last_nbr, nbr, agent_node, out=out, col0=out_col)
        if out is not None:
            return out
        R = N if agent_node is None else agent_node.shape[1]
        return res.reshape(B, R, -1)

    def forward(self, x, mask, node_agent_matrix=None, max_degree=None, no_agent_mapping=False):
        # the neighbour table holds every neighbour (aggregation always uses the full mask,
        # src/model.py:582-593); max_degree only sizes the readout: below the true degree the
        # reference's _get_neighbor_h fails, above it the extra slots read zeros (-1 columns,
        # which the aggregate skips)
        nbr = dense_to_nbr(mask)
        if max_degree is not None:
            md = int(max_degree)
            if md < nbr.shape[-1]:
                raise ValueError(f"max_degree {md} is below the largest node degree {nbr.shape[-1]} of the batch")
            if md > nbr.shape[-1]:
                nbr = F.pad(nbr, (0, md - nbr.shape[-1]), value=-1).contiguous()
        an = None if (no_agent_mapping or node_agent_matrix is None) else node_agent_to_index(node_agent_matrix)
        return self.forward_graph(x, nbr, an)

    @staticmethod
    def output_to_network_obs(netmon_out, node_agent_matrix):
        return torch.bmm(netmon_out.transpose(1, 2), node_agent_matrix).transpose(1, 2)


class Q_Net(nn.Module):
    def __init__(self, in_features, actions):
        super().__init__()
        self.fc = Linear(in_features, actions, act=0)

    def forward(self, x):
        return self.fc(x)


class DQN(nn.Module):
    """src/model.py:187-203: MLP encoder (activation on output) + linear Q head."""

    def __init__(self, in_features, mlp_units, num_actions, activation="leaky_relu"):
        super().__init__()
        self.encoder = MLP(in_features, mlp_units, activation=activation)
        self.q_net = Q_Net(self.encoder.out_features, num_actions)

    def forward(self, x, mask=None):
        return self.q_net(self.encoder(x))

    def forward_split(self, env_obs, graph_obs):
        """forward(joint_obs(env_obs, graph_obs)) without the joint tensor: the first layer reads the
        env observation [B, A, od] (rows padded to 16 bytes, e.g. replay batches) and the NetMon
        graph observation [B, A, G] as two GEMM sources (_JointLinearFn)."""
        B, A, od = env_obs.shape
        e2 = env_obs.reshape(B * A, od)
        g2 = graph_obs.reshape(B * A, graph_obs.shape[-1])
        layers = self.encoder.linear_layers
        if not joint_first_layer_ok(g2, e2) or layers[0].in_features != od + g2.shape[1]:
            from .train import joint_obs

            return self(joint_obs(env_obs, graph_obs))
        lin = layers[0]
        h = _JointLinearFn.apply(g2, e2, lin.weight, lin.bias, lin)
        for lin in layers[1:]:
            h = lin(h)
        return self.q_net(h).view(B, A, -1)

    def forward_rows(self, x2d, ldx, k, scratch, **unused):
        """no-grad fast path: q [rows, actions] from a strided observation buffer; the last
        hidden layer and the Q head run as one kernel (gm_gemm_x3_head) when they fit it."""
        from . import fused as FU

        layers = self.encoder.linear_layers
        out = scratch(len(layers), x2d.shape[0], self.q_net.fc.out_features)
        if len(layers) > 1 and FU.head_ok(layers[-1], self.q_net.fc):
            h = self.encoder.forward_into(x2d, ldx, k, scratch, n_layers=len(layers) - 1)
            return FU.linear_head(layers[-1], self.q_net.fc, h, h.stride(0), h.shape[1], out)
        h = self.encoder.forward_into(x2d, ldx, k, scratch)
        return linear_raw(h, h.stride(0), h.shape[1], self.q_net.fc.weight, self.q_net.fc.bias, 0, out=out,
                          ldy=out.stride(0), wcache=self.q_net.fc._wc, tag=self.q_net.fc.tag)


def tag_modules(root, prefix=""):
    """Name every Linear/LSTMCell by its module path (kernel timer tags)."""
    for name, m in root.named_modules():
        if isinstance(m, (Linear, LSTMCell, LayerNormLSTMCell, GRUCell)):
            m.tag = prefix + name


# ---------------------------------------------------------------------------
# Agent models of the reference besides DQN: DGN (agent attention), DQNR (recurrent
# DQN), CommNet (recurrent + masked mean communication), src/model.py:45-184, 653-794.
# forward(x, mask) is the reference signature (autograd; the GEMMs on the MFMA kernels,
# the small A x A attention / communication in torch). forward_rows() is the no-grad
# rollout path: fused GEMMs + gm_agent_attention / gm_agent_comm, no A x A tensors in torch.
# ---------------------------------------------------------------------------
def _adj_i8(mask):
    return mask.contiguous() if mask.dtype == torch.int8 else (mask != 0).to(torch.int8).contiguous()


class AttModel(nn.Module):
    """src/model.py:45-117: v/k/q = act(linear(x)) per head, softmax(q k^T / sqrt(dk))
    masked by the agent adjacency (-1e9), att v + v, heads concatenated, act(fc_out).
    forward returns (out, att_weights) with the weights before masking, like the reference."""

    def __init__(self, in_features, k_features, v_features, out_features, num_heads, activation="leaky_relu"):
        super().__init__()
        self.k_features, self.v_features, self.num_heads = k_features, v_features, num_heads
        act = act_code(activation)  # the reference's DGN passes activation_fn as both vkq and output act
        self.fc_v = Linear(in_features, v_features * num_heads, act=act)
        self.fc_k = Linear(in_features, k_features * num_heads, act=act)
        self.fc_q = Linear(in_features, k_features * num_heads, act=act)
        self.fc_out = Linear(v_features * num_heads, out_features, act=act)
        self.attention_scale = 1 / (k_features ** 0.5)

    def forward(self, x, mask):
        B, A = x.shape[0], x.shape[1]
        nh = self.num_heads
        v = self.fc_v(x).view(B, A, nh, self.v_features).transpose(1, 2)
        q = self.fc_q(x).view(B, A, nh, self.k_features).transpose(1, 2)
        k = self.fc_k(x).view(B, A, nh, self.k_features).transpose(1, 2)
        att_weights = torch.matmul(q, k.transpose(2, 3)) * self.attention_scale
        att = F.softmax(att_weights.masked_fill(mask.unsqueeze(1) == 0, -1e9), dim=-1)
        out = (torch.matmul(att, v) + v).transpose(1, 2).contiguous().view(B, A, -1)
        return self.fc_out(out), att_weights

    def forward_rows(self, x2d, ldx, adj, B, A, out, ldo, scratch, att_weights=None):
        """no-grad: rows [B*A] of x (stride ldx) -> out rows (stride ldo) via one q/k/v GEMM,
        gm_agent_attention and the fc_out GEMM."""
        from . import fused as FU

        M = B * A
        nh, dk, dv = self.num_heads, self.k_features, self.v_features
        qkv = scratch(("qkv", id(self)), M, nh * (dv + 2 * dk))
        FU.linear_rows(FU.concat_linears(self, (self.fc_v, self.fc_k, self.fc_q)), x2d, ldx, M, qkv, qkv.stride(0))
        core = scratch(("att", id(self)), M, nh * dv)
        vo, ko, qo = 0, nh * dv, nh * (dv + dk)
        L.check(L.lib().gm_agent_attention(
            qkv.data_ptr() + 4 * qo, qkv.data_ptr() + 4 * ko, qkv.data_ptr() + 4 * vo, qkv.stride(0), L.ptr(adj), B, A,
            nh, dk, dv, L.ptr(core), core.stride(0), L.ptr(att_weights), _s()))
        FU.linear_rows(self.fc_out, core, core.stride(0), M, out, ldo)
        return out


class DGN(nn.Module):
    """src/model.py:120-176 "Graph Convolutional Reinforcement Learning": MLP encoder,
    num_attention_layers AttModel layers (dk = dv = 16), Q head on the concatenation of
    the encoder output and every attention layer's output. att_weights holds the
    per-layer weights of the last forward (attention regularisation, src/main.py:924-954)."""

    def __init__(self, in_features, mlp_units, num_actions, num_heads=8, num_attention_layers=2,
                 activation="leaky_relu"):
        super().__init__()
        self.encoder = MLP(in_features, mlp_units, activation=activation)
        hidden = self.encoder.out_features
        self.att_layers = nn.ModuleList(
            [AttModel(hidden, 16, 16, hidden, num_heads, activation) for _ in range(num_attention_layers)])
        self.q_net = Q_Net(hidden * (num_attention_layers + 1), num_actions)
        self.att_weights = []

    def forward(self, x, mask):
        h = self.encoder(x)
        q_input = h
        self.att_weights.clear()
        for layer in self.att_layers:
            if torch.is_grad_enabled() or x.shape[1] > 64:
                h, w = layer(h, mask)
            else:  # no-grad: the HIP attention core (weights recorded for the regulariser)
                B, A, Hd = h.shape
                w = torch.empty(B, layer.num_heads, A, A, device=x.device)
                o = torch.empty(B * A, layer.fc_out.out_features, device=x.device)
                hr = h.reshape(B * A, Hd).contiguous()
                layer.forward_rows(hr, hr.stride(0), _adj_i8(mask), B, A, o, o.stride(0), _scratch_dict({}), w)
                h = o.view(B, A, -1)
            self.att_weights.append(w)
            q_input = torch.cat((q_input, h), dim=-1)
        return self.q_net(q_input)

    def forward_rows(self, x2d, ldx, k, scratch, adj=None, B=None, A=None):
        """no-grad rollout path: encoder, attention layers and Q head over a strided
        observation buffer; [h_enc | h_1 | ...] are written side by side (no concat)."""
        from . import fused as FU

        M = x2d.shape[0]
        hid = self.encoder.out_features
        nl = len(self.att_layers)
        qin = scratch(("dgn_qin", id(self)), M, hid * (nl + 1))
        FU.mlp_rows(self.encoder, x2d, ldx, k, M, scratch, out=qin, ldo=qin.stride(0))
        for li, layer in enumerate(self.att_layers):
            layer.forward_rows(qin[:, li * hid:], qin.stride(0), adj, B, A, qin[:, (li + 1) * hid:], qin.stride(0),
                               scratch)
        out = scratch(("dgn_q", id(self)), M, self.q_net.fc.out_features)
        FU.linear_rows(self.q_net.fc, qin, qin.stride(0), M, out, out.stride(0))
        return out


def _scratch_dict(d):
    def get(key, m, n):
        b = d.get((key, m, n))
        if b is None:
            b = torch.empty(m, n, device="cuda")
            d[(key, m, n)] = b
        return b
    return get


class DQNR(nn.Module):
    """src/model.py:653-744: MLP encoder, LSTMCell over the encoding with a carried agent
    state, Q head. `state` is [B, A, 2H] ([h | c] per agent) or None (= zeros) between
    calls, like the reference's external layout (_state_reshape_out)."""

    def __init__(self, in_features, mlp_units, num_actions, activation="leaky_relu"):
        super().__init__()
        self.encoder = MLP(in_features, mlp_units, activation=activation)
        H = self.encoder.out_features
        self.lstm = LSTMCell(H, H)
        self.state = None
        self.q_net = Q_Net(H, num_actions)

    def get_state_len(self):
        return 2 * self.lstm.hidden_size

    def _split(self, B, A):
        H = self.lstm.hidden_size
        if self.state is None:
            z = torch.zeros(B * A, H, device=self.lstm.weight_ih.device)
            return z, z
        st = self.state.reshape(B * A, 2, H)
        return st[:, 0], st[:, 1]

    def _step(self, x, h, c, B, A):
        h1, c1 = self.lstm(x, (h.contiguous(), c.contiguous()))
        return h1, c1

    def forward(self, x, mask=None):
        B, A, _ = x.shape
        h = self.encoder(x).reshape(B * A, -1)
        hs, cs = self._split(B, A)
        h1, c1 = self._step(h, hs, cs, B, A)
        self.state = torch.stack((h1, c1), 1).reshape(B, A, -1)
        return self.q_net(h1.view(B, A, -1))

    def _lstm_rows(self, x, ldx, S_in, S_out, M):
        """fused LSTM GEMM: S_out = [h' | c'] rows from x rows and S_in = [h | c] rows."""
        from . import fused as FU

        H = self.lstm.hidden_size
        wp, ldw, bp, x3 = FU.pack_lstm(self.lstm)
        FU.gemm(FU.dense(x.data_ptr(), ldx, H), FU.dense(S_in.data_ptr(), S_in.stride(0), H), wp.data_ptr(), ldw,
                bp.data_ptr(), M, 4 * H, FU.GM_EPI_LSTM, S_out.data_ptr(), S_out.stride(0),
                S_out.data_ptr() + 4 * H, S_out.stride(0), S_in.data_ptr() + 4 * H, S_in.stride(0),
                tag=self.lstm.tag and f"lstm:{self.lstm.tag}:{M}x{4 * H}x{2 * H}", x3=x3)

    def _state_rows(self, B, A, M):
        if self.state is None:
            return torch.zeros(M, 2 * self.lstm.hidden_size, device=self.lstm.weight_ih.device)
        return self.state.reshape(M, -1).contiguous()

    def forward_rows(self, x2d, ldx, k, scratch, adj=None, B=None, A=None):
        from . import fused as FU

        M = x2d.shape[0]
        h = FU.mlp_rows(self.encoder, x2d, ldx, k, M, scratch)
        S = torch.empty(M, 2 * self.lstm.hidden_size, device=x2d.device)
        self._lstm_rows(h, h.stride(0), self._state_rows(B, A, M), S, M)
        self.state = S.view(B, A, -1)
        out = scratch(("q", id(self)), M, self.q_net.fc.out_features)
        FU.linear_rows(self.q_net.fc, S, S.stride(0), M, out, out.stride(0), k=self.lstm.hidden_size)
        return out


class CommNet(DQNR):
    """src/model.py:747-794: DQNR whose hidden state is, for comm_rounds rounds, added to
    the mean of the other adjacent agents' hidden states (self excluded, count clamped to
    1) and fed through the LSTM again as both input and hidden state (cell states are not
    communicated, as in IC3Net)."""

    def __init__(self, in_features, mlp_units, num_actions, comm_rounds=2, activation="leaky_relu"):
        super().__init__(in_features, mlp_units, num_actions, activation)
        assert comm_rounds >= 0
        self.comm_rounds = comm_rounds

    def forward(self, x, mask):
        B, A, _ = x.shape
        h = self.encoder(x).reshape(B * A, -1)
        hs, cs = self._split(B, A)
        h, c = self._step(h, hs, cs, B, A)
        m = (mask != 0).float() * ~torch.eye(A, dtype=torch.bool, device=x.device).unsqueeze(0)
        cnt = torch.clamp(m.sum(dim=-1).unsqueeze(-1), min=1)
        for _ in range(self.comm_rounds):
            hv = h.view(B, A, -1)
            hv = hv + torch.bmm(m, hv) / cnt
            h = hv.reshape(B * A, -1)
            h, c = self._step(h, h, c, B, A)
        self.state = torch.stack((h, c), 1).reshape(B, A, -1)
        return self.q_net(h.view(B, A, -1))

    def forward_rows(self, x2d, ldx, k, scratch, adj=None, B=None, A=None):
        from . import fused as FU

        M = x2d.shape[0]
        H = self.lstm.hidden_size
        h = FU.mlp_rows(self.encoder, x2d, ldx, k, M, scratch)
        S = torch.empty(M, 2 * H, device=x2d.device)
        self._lstm_rows(h, h.stride(0), self._state_rows(B, A, M), S, M)
        for _ in range(self.comm_rounds):
            hc = torch.empty(M, 2 * H, device=x2d.device)  # [h + comm | c]
            L.check(L.lib().gm_agent_comm(L.ptr(S), S.stride(0), L.ptr(adj), B, A, H, L.ptr(hc), hc.stride(0), _s()))
            hc[:, H:].copy_(S[:, H:])
            S2 = torch.empty(M, 2 * H, device=x2d.device)
            self._lstm_rows(hc, hc.stride(0), hc, S2, M)
            S = S2
        self.state = S.view(B, A, -1)
        out = scratch(("q", id(self)), M, self.q_net.fc.out_features)
        FU.linear_rows(self.q_net.fc, S, S.stride(0), M, out, out.stride(0), k=H)
        return out
