"""Fused no-grad rollout path over gm_gemm_f32 (include/graph_marl_amd.h).

NetMon step (reference src/model.py:476-580):
  x  = MLP encoder(node_obs)              gm_routing_node_encoder (layer 0) + gm_linear_f32 x2
  S1 = LSTM_obs([x | h_state], c_state)                        one GEMM, gate math in epilogue
  S2 = LSTM_upd([Σ_{I+A} h(S1) | h(S1)], c(S1))  (K times)     aggregate folded into the A load
state = S_K ([h | c] per node, the reference's (B, N, 2H) layout), h_prev = h before the
last update (readout's neighbour features, src/model.py:510-519).

DQN Q (src/model.py:187-203) on the joint observation without materialising it:
  h1 = leaky(W1 @ [readout(h_final, h_prev, nbr, agent_node) | env_obs] + b1)
so the NetMon readout + agent gather (src/model.py:582-631) happen in the GEMM's A load.
Weights are packed once per parameter version (LSTM gate interleave, W1 column order,
and for the split-f16 form (L.GEMM_MODE == "x3", gm_gemm_x3) the hi/lo f16 split).
"""
import ctypes as C

import torch
import torch.nn.functional as F

from . import _lib as L

GM_A_DENSE, GM_A_AGGREGATE, GM_A_READOUT, GM_A_ROUTING_ENC = 0, 1, 2, 3
GM_EPI_BIAS, GM_EPI_BIAS_LEAKY, GM_EPI_LSTM, GM_EPI_GRU = 0, 1, 2, 3


def _epi(act):
    """bias + activation epilogue code of a layer's GM_ACT_* code (model.epi_code)."""
    from .model import epi_code

    return epi_code(act)

# LSTM update cell: a strided aggregate pass (gm_mp_aggregate_rows, 26-29 us at 81920 nodes) +
# the cell on dense [Σ h | h] (103-111 us) instead of the AGGREGATE A source inside the GEMM
# (159 us); False selects the in-GEMM aggregate
PRE_AGG = True


class ASrc(C.Structure):
    _fields_ = [
        ("mode", C.c_int32), ("p0", C.c_void_p), ("p1", C.c_void_p), ("ld0", C.c_int64), ("ld1", C.c_int64),
        ("nbr", C.c_void_p), ("agent_node", C.c_void_p), ("n_nodes", C.c_int32), ("deg", C.c_int32),
        ("mean", C.c_int32), ("rows_per_graph", C.c_int32), ("k", C.c_int32), ("hidden", C.c_int32),
        ("scale", C.c_void_p), ("amax", C.c_void_p), ("bias0", C.c_void_p), ("act0", C.c_int32),
    ]


def _setup():
    lib = L.lib()
    if not getattr(lib, "_gemm_ready", False):
        vp = C.c_void_p
        lib.gm_gemm_f32.argtypes = [C.POINTER(ASrc), C.POINTER(ASrc), vp, C.c_int64, vp, C.c_int32, C.c_int32,
                                    C.c_int32, vp, C.c_int64, vp, C.c_int64, vp, C.c_int64, vp, vp]
        lib.gm_gemm_x3.argtypes = [C.POINTER(ASrc), C.POINTER(ASrc), vp, vp, vp, C.c_int32, C.c_int32,
                                   C.c_int32, vp, C.c_int64, vp, C.c_int64, vp, C.c_int64, vp, vp]
        lib.gm_absmax_scale.argtypes = [vp, C.c_int64, vp, vp]
        lib.gm_absmax_finish.argtypes = [vp, vp]
        lib.gm_absmax_scale_rows.argtypes = [vp, C.c_int64, C.c_int32, C.c_int64, vp, vp]
        lib.gm_gemm_x3_wgrad.argtypes = [vp, C.c_int64, vp, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                         vp, vp, vp, C.c_int64, vp]
        lib.gm_gemm_x3_wgrad2.argtypes = [vp, C.c_int64, C.POINTER(L.WgradSrc), C.c_int32, C.POINTER(L.WgradSrc),
                                          C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, vp, C.c_int64, vp]
        lib.gm_gemm_x3_head.argtypes = [C.POINTER(ASrc), vp, vp, vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int64,
                                        vp, C.c_int32, vp, C.c_int64, vp, C.c_int64, vp]
        lib.gm_gemm_x3_dgrad.argtypes = [C.POINTER(ASrc), vp, vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int64, vp,
                                         C.c_int64, vp, C.c_int64, vp, vp, vp]
        i32, i64 = C.c_int32, C.c_int64
        lib.gm_encoder_x3.argtypes = [C.POINTER(ASrc), vp, vp, vp, i32, vp, vp, vp, i32, i32, i32, i32, vp, i64, vp]
        lib._gemm_ready = True
    return lib


class X3:
    """Weights split for gm_gemm_x3: packed hi/lo f16 blocks + the device scalar 1/S."""
    __slots__ = ("wp", "sinv", "n", "k")

    def __init__(self, w, ldw, n, k):
        lib = _setup()
        nb = lib.gm_gemm_pack_x3_bytes(n, k)
        self.wp = torch.empty(nb, dtype=torch.uint8, device=w.device)
        self.sinv = torch.empty(1, dtype=torch.float32, device=w.device)
        self.n, self.k = n, k
        L.check(lib.gm_gemm_pack_x3(w.data_ptr(), ldw, n, k, self.wp.data_ptr(), self.sinv.data_ptr(),
                                    L.stream_ptr()))


def use_x3(n):
    """The split-f16 form runs every GEMM wider than the 32-column tail (the Q head stays f32)."""
    return L.GEMM_MODE == "x3" and n > 32


def dense(p, ld, k, scale=None, amax=None):
    """DENSE A source; scale: device float from gm_absmax_scale; amax: zeroed device float that
    receives max|A| as float bits (gm_absmax_finish turns it into the scale); split-f16 only."""
    s = ASrc()
    s.mode, s.p0, s.ld0, s.k = GM_A_DENSE, p, ld, k
    s.scale = scale
    s.amax = amax
    return s


def routing_enc_src(lin, x, nbr, N):
    """ROUTING_ENC A source (gm_gemm_x3): the NetMon encoder's first layer `lin` on routing node
    observations x [G*N, >= 4N+8] computed inside the next layer's A-tile load (no m x k output)."""
    if not hasattr(lin, "_packed_t"):
        lin._packed_t = Packed()
    wt = lin._packed_t.get(_key(lin.weight), lambda: lin.weight.detach().t().contiguous())
    s = ASrc()
    s.mode, s.p0, s.ld0, s.p1, s.ld1 = GM_A_ROUTING_ENC, x.data_ptr(), x.stride(0), wt.data_ptr(), wt.stride(0)
    s.nbr, s.n_nodes, s.deg, s.k = nbr.data_ptr(), N, 3, lin.out_features
    s.bias0 = None if lin.bias is None else lin.bias.data_ptr()
    s.act0 = lin.act
    return s


# the rollout folds the NetMon encoder's first layer into the second layer's A-tile load when the split
# form runs and 4N + 8 <= 208, N <= 50 (GM_A_ROUTING_ENC, always on 16x16x32 MFMA); otherwise
# gm_routing_node_encoder + a DENSE second layer (tests set it False to compare the two forms)
RENC_FOLD = True


def renc_fold_ok(layers, N, Fd, nbr):
    return (RENC_FOLD and L.GEMM_MODE == "x3" and len(layers) >= 2 and routing_encoder_ok(layers[0], N, Fd, nbr)
            and 4 * N + 8 <= 208 and layers[0].out_features % 32 == 0 and layers[0].out_features <= 1024
            and use_x3(layers[1].out_features) and layers[1].in_features == layers[0].out_features
            and layers[1].bias is not None)


# the rollout's NetMon encoder [4N+8 -> k -> 256 -> 128] (the CLI default 512, 256 with H = 128) in one launch
# (gm_encoder_x3: layer 2's output stays on chip for layer 3); other shapes run the fold + a layer-3 GEMM
ENC_CHAIN = True


def encoder_chain_ok(layers, N, Fd, nbr):
    return (ENC_CHAIN and len(layers) >= 3 and renc_fold_ok(layers, N, Fd, nbr) and layers[1].out_features == 256
            and layers[2].in_features == 256 and layers[2].out_features == 128 and layers[1].bias is not None
            and layers[2].bias is not None and use_x3(128))


def encoder_chain(l0, l1, l2, x, nbr, N, out):
    """out = l2(l1(l0(x))) on routing node observations in one launch (gm_encoder_x3)."""
    lib = _setup()
    x1, x2 = pack_x3(l1), pack_x3(l2)
    M = x.shape[0]
    with L.timed(l1.tag and f"linear:{l1.tag}+chain:{M}x{l1.out_features}x{l1.in_features}"):
        L.check(lib.gm_encoder_x3(C.byref(routing_enc_src(l0, x, nbr, N)), x1.wp.data_ptr(), x1.sinv.data_ptr(),
                                  l1.bias.data_ptr(), l1.act, x2.wp.data_ptr(), x2.sinv.data_ptr(), l2.bias.data_ptr(),
                                  l2.act, M, l1.out_features, l2.out_features, out.data_ptr(), out.stride(0),
                                  L.stream_ptr()))
    return out


def aggregate(p, ld, k, nbr, n_nodes, mean=False):
    s = ASrc()
    s.mode, s.p0, s.ld0, s.k = GM_A_AGGREGATE, p, ld, k
    s.nbr, s.n_nodes, s.deg, s.mean = nbr.data_ptr(), n_nodes, nbr.shape[-1], int(mean)
    return s


def readout(h_final, ld_f, h_prev, ld_p, nbr, agent_node, n_nodes, hidden):
    s = ASrc()
    s.mode, s.p0, s.ld0, s.p1, s.ld1 = GM_A_READOUT, h_final, ld_f, h_prev, ld_p
    s.nbr, s.agent_node, s.n_nodes, s.deg = nbr.data_ptr(), agent_node.data_ptr(), n_nodes, nbr.shape[-1]
    s.rows_per_graph, s.hidden, s.k = agent_node.shape[-1], hidden, (nbr.shape[-1] + 1) * hidden
    return s


def gemm(a0, a1, w, ldw, b, m, n, epi, y, ldy, y2=None, ldy2=0, c_in=None, ldc=0, act_out=None, tag=None, x3=None):
    """y = epi(A @ W^T + b); with x3 (an X3 of the same W) the split-f16 form runs."""
    lib = _setup()
    a1p = None if a1 is None else C.byref(a1)
    with L.timed(tag):
        if x3 is not None:
            assert x3.n == n and x3.k == a0.k + (0 if a1 is None else a1.k), "packed weights do not match the GEMM"
            L.check(lib.gm_gemm_x3(C.byref(a0), a1p, x3.wp.data_ptr(), x3.sinv.data_ptr(), b, m, n, epi, y, ldy,
                                   y2, ldy2, c_in, ldc, act_out, L.stream_ptr()))
        else:
            L.check(lib.gm_gemm_f32(C.byref(a0), a1p, w, ldw, b, m, n, epi, y, ldy, y2, ldy2, c_in, ldc, act_out,
                                    L.stream_ptr()))


def _key(*ts):
    return tuple((t.data_ptr(), t._version) for t in ts)


class Packed:
    """Per-module cache of packed weights, refreshed when a parameter changes; safe to share
    between streams (L.Published)."""

    def __init__(self):
        self.key = None
        self.val = None
        self.pub = None

    def get(self, key, fn):
        if key != self.key:
            self.val = fn()
            self.key = key
            self.pub = L.Published()
        else:
            self.pub.acquire(self.val)
        return self.val

    def __deepcopy__(self, memo):
        return Packed()  # a copied module (target network) packs its own parameters


def _pad_cols(w):
    k = w.shape[1]
    kp = (k + 3) // 4 * 4
    return F.pad(w, (0, kp - k)).contiguous(), kp


def pack_lstm(cell):
    """[W_ih | W_hh] with rows interleaved per 32 hidden units: row 128t + 32g + u holds gate g
    of unit 32t + u (original row g*H + 32t + u); bias b_ih + b_hh in the same order."""
    if not hasattr(cell, "_packed"):
        cell._packed = Packed()

    def build():
        with torch.no_grad():
            H = cell.hidden_size
            assert H % 32 == 0, "fused LSTM needs H % 32 == 0"
            w = torch.cat([cell.weight_ih, cell.weight_hh], 1)
            b = cell.bias_ih + cell.bias_hh
            t = torch.arange(H // 32, device=w.device)
            g = torch.arange(4, device=w.device)
            u = torch.arange(32, device=w.device)
            orig = (g[None, :, None] * H + 32 * t[:, None, None] + u[None, None, :]).reshape(-1)
            wp, ldw = _pad_cols(w[orig])
            x3 = X3(wp, ldw, 4 * H, 2 * H) if use_x3(4 * H) else None
            return wp, ldw, b[orig].contiguous(), x3

    return cell._packed.get(_key(cell.weight_ih, cell.weight_hh, cell.bias_ih, cell.bias_hh) + (L.GEMM_MODE,), build)


def _interleave(w, b, H):
    """Rows of a gate-major [4H, K] matrix (gates g = 0..3 of H rows) in the gate-tile order of the
    LSTM/GRU epilogues: row 128t + 32g + u holds gate g of unit 32t + u."""
    t = torch.arange(H // 32, device=w.device)
    g = torch.arange(4, device=w.device)
    u = torch.arange(32, device=w.device)
    orig = (g[None, :, None] * H + 32 * t[:, None, None] + u[None, None, :]).reshape(-1)
    return w[orig], b[orig]


def pack_gru(cell):
    """torch.nn.GRUCell (r, z, n) as four gate tiles on A = [x | h] for GM_EPI_GRU: r and z rows
    [W_ih | W_hh], n_x rows [W_in | 0], n_h rows [0 | W_hn] (W_hn h stays apart for r * (W_hn h +
    b_hn)); biases b_ir + b_hr, b_iz + b_hz, b_in, b_hn."""
    if not hasattr(cell, "_packed"):
        cell._packed = Packed()

    def build():
        with torch.no_grad():
            H = cell.hidden_size
            assert H % 32 == 0, "fused GRU needs H % 32 == 0"
            wi, wh, bi, bh = cell.weight_ih, cell.weight_hh, cell.bias_ih, cell.bias_hh
            z = torch.zeros(H, H, device=wi.device)
            w = torch.cat([torch.cat([wi[:2 * H], wh[:2 * H]], 1), torch.cat([wi[2 * H:], z], 1),
                           torch.cat([z, wh[2 * H:]], 1)], 0)
            b = torch.cat([bi[:2 * H] + bh[:2 * H], bi[2 * H:], bh[2 * H:]])
            w, b = _interleave(w, b, H)
            wp, ldw = _pad_cols(w)
            x3 = X3(wp, ldw, 4 * H, 2 * H) if use_x3(4 * H) else None
            return wp, ldw, b.contiguous(), x3

    return cell._packed.get(_key(cell.weight_ih, cell.weight_hh, cell.bias_ih, cell.bias_hh) + (L.GEMM_MODE,), build)


def pack_lnlstm(cell):
    """LayerNormLSTMCell: W_ih and W_hh as two separate GEMM weights (each product gets its own
    LayerNorm before they are summed), split-f16 packs when that form runs."""
    if not hasattr(cell, "_packed"):
        cell._packed = Packed()

    def build():
        with torch.no_grad():
            H = cell.hidden_size
            out = []
            for w in (cell.weight_ih, cell.weight_hh):
                wp, ldw = _pad_cols(w)
                out.append((wp, ldw, X3(wp, ldw, 4 * H, w.shape[1]) if use_x3(4 * H) else None))
            return out

    return cell._packed.get(_key(cell.weight_ih, cell.weight_hh) + (L.GEMM_MODE,), build)


def fold_env_weight(we, n):
    """Env-obs weight columns [out, 6N+10] -> [out, 6N+8] for the GEMM-ready obs copy
    (gm_obs_buffers.obs_gemm), exact in real arithmetic (src/env/routing.py:269-315 rows):
    position one-hot column N-1 = sum(target one-hot) - sum(position one-hots 0..N-2), and the
    edge flag (column 2N) = sum of the next-hop one-hot (columns 2N+1..3N). Summed in fp64,
    rounded once."""
    w = we.double()
    last, flag = w[:, n - 1:n], w[:, 2 * n:2 * n + 1]
    out = torch.cat([w[:, :n - 1] - last, w[:, n:2 * n] + last, w[:, 2 * n + 1:3 * n + 1] + flag, w[:, 3 * n + 1:]], 1)
    return out.to(we.dtype)


def pack_dqn_first(lin, obs_dim, fold_n=None):
    """W1 columns reordered to [graph part | env obs part] to match A = [readout | env obs];
    fold_n = N: env part folded to the 6N+8 columns of the GEMM-ready obs copy."""
    if not hasattr(lin, "_packed_first"):
        lin._packed_first = Packed()

    def build():
        with torch.no_grad():
            we = lin.weight[:, :obs_dim]
            if fold_n is not None:
                we = fold_env_weight(we, fold_n)
            w = torch.cat([lin.weight[:, obs_dim:], we], 1).contiguous()
            wp, ldw = _pad_cols(w)
            n = lin.out_features
            x3 = X3(wp, ldw, n, w.shape[1]) if use_x3(n) else None
            return wp, ldw, lin.bias.contiguous(), x3

    return lin._packed_first.get(_key(lin.weight, lin.bias) + (obs_dim, fold_n, L.GEMM_MODE), build)


def pack_x3(lin):
    """Split-f16 weights of a Linear (None when the f32 form runs it)."""
    if not use_x3(lin.out_features):
        return None
    if not hasattr(lin, "_packed_x3"):
        lin._packed_x3 = Packed()
    return lin._packed_x3.get(_key(lin.weight), lambda: X3(lin.weight, lin.weight.stride(0), lin.out_features,
                                                           lin.in_features))


def head_ok(lin, fc):
    """The last hidden layer and the Q head run as one kernel (gm_gemm_x3_head) in the split
    form when the layer is at most 256 wide and the head at most 4 outputs, both with bias."""
    return (use_x3(lin.out_features) and lin.out_features <= 256 and fc.out_features <= 4 and fc.act == 0
            and fc.in_features == lin.out_features and lin.bias is not None and fc.bias is not None)


def linear_head(lin, fc, x, ldx, k, q, y=None):
    """q = fc(act(x @ W^T + b)) without writing the hidden activation (written to y if given)."""
    lib = _setup()
    x3 = pack_x3(lin)
    M = q.shape[0]
    wq = fc.weight if fc.weight.is_contiguous() else fc.weight.contiguous()
    tag = lin.tag and f"linear:{lin.tag}+head:{M}x{lin.out_features}x{k}"
    with L.timed(tag):
        L.check(lib.gm_gemm_x3_head(C.byref(dense(x.data_ptr(), ldx, k)), x3.wp.data_ptr(), x3.sinv.data_ptr(),
                                    lin.bias.data_ptr(), M, lin.out_features, lin.act, wq.data_ptr(),
                                    wq.stride(0), fc.bias.data_ptr(), fc.out_features, q.data_ptr(), q.stride(0),
                                    None if y is None else y.data_ptr(), 0 if y is None else y.stride(0),
                                    L.stream_ptr()))
    return q


def _linear(x, ldx, k, lin, out):
    wp, ldw = lin._wc.get(lin.weight)
    a = dense(x.data_ptr(), ldx, k)
    gemm(a, None, wp.data_ptr(), ldw, lin.bias.data_ptr(), x.shape[0], lin.out_features,
         _epi(lin.act), out.data_ptr(), out.stride(0),
         tag=lin.tag and f"linear:{lin.tag}:{x.shape[0]}x{lin.out_features}x{k}", x3=pack_x3(lin))
    return out


def linear_rows(lin, x, ldx, M, out, ldo, k=None):
    """out rows (stride ldo) = act(x rows (stride ldx, first k = in_features columns) @ W^T + b)."""
    k = lin.in_features if k is None else k
    wp, ldw = lin._wc.get(lin.weight)
    gemm(dense(x.data_ptr(), ldx, k), None, wp.data_ptr(), ldw, lin.bias.data_ptr(), M, lin.out_features,
         _epi(lin.act), out.data_ptr(), ldo,
         tag=lin.tag and f"linear:{lin.tag}:{M}x{lin.out_features}x{k}", x3=pack_x3(lin))
    return out


def mlp_rows(mlp, x, ldx, k, M, scratch, out=None, ldo=None):
    """MLP over strided rows; the last layer writes into `out` (stride ldo) when given.
    Rows whose stride or base is not 16-byte aligned are first copied into a padded buffer."""
    if ldx % 4 or x.data_ptr() % 16:
        xp = scratch(("mlp_in", id(mlp)), M, (k + 3) // 4 * 4)
        xp[:, :k].copy_(torch.as_strided(x, (M, k), (ldx, 1)))
        x, ldx = xp, xp.stride(0)
    h, ld, kk = x, ldx, k
    layers = list(mlp.linear_layers)
    for i, lin in enumerate(layers):
        if i == len(layers) - 1 and out is not None:
            dst, ldd = out, ldo
        else:
            dst = scratch(("mlp", id(mlp), i), M, lin.out_features)
            ldd = dst.stride(0)
        linear_rows(lin, h, ld, M, dst, ldd, k=kk)
        h, ld, kk = dst, ldd, lin.out_features
    return h


class _CatLinear:
    """Row-concatenation of Linears with the same input and activation (one GEMM)."""

    def __init__(self, linears):
        from .model import _WeightCache

        with torch.no_grad():
            self.weight = torch.cat([l.weight for l in linears], 0).contiguous()
            self.bias = torch.cat([l.bias for l in linears], 0).contiguous()
        self.act = linears[0].act
        assert all(l.act == self.act for l in linears)
        self.in_features = linears[0].in_features
        self.out_features = self.weight.shape[0]
        self._wc = _WeightCache()
        self.tag = linears[0].tag and linears[0].tag.rsplit(".", 1)[0] + ".fc_vkq"


def concat_linears(owner, linears):
    """Cached _CatLinear of `linears` (rebuilt when a parameter changes)."""
    if not hasattr(owner, "_packed_cat"):
        owner._packed_cat = Packed()
    key = tuple(x for l in linears for x in _key(l.weight, l.bias)) + (L.GEMM_MODE,)
    return owner._packed_cat.get(key, lambda: _CatLinear(linears))


def routing_encoder_ok(lin, N, Fd, nbr):
    """The routing node-obs layout (4N+8 columns, degree-3 neighbour table) lets the first
    encoder layer run as a 12-column gather (gm_routing_node_encoder)."""
    return (Fd == 4 * N + 8 and nbr.shape[-1] == 3 and lin.out_features % 64 == 0 and
            (4 * N + 8) * 64 * (2 if lin.out_features % 128 == 0 and (4 * N + 8) <= 128 else 1) * 4 <= 65536)


def routing_encoder(lin, x, nbr, G, N, out, sbits=None, act=None):
    """y = act(W x + b) on routing node observations from their nonzero entries; sbits (optional,
    int32 [rows][ceil(n / 32)]) receives the sign bits of y (the training backward's leaky mask);
    act overrides lin.act (0: the pre-activation)."""
    if not hasattr(lin, "_packed_t"):
        lin._packed_t = Packed()
    wt = lin._packed_t.get(_key(lin.weight), lambda: lin.weight.detach().t().contiguous())
    with L.timed(lin.tag and f"routing_enc:{lin.tag}:{G * N}x{lin.out_features}"):
        L.check(L.lib().gm_routing_node_encoder_bits(L.ptr(x), x.stride(0), L.ptr(nbr), G, N, L.ptr(wt),
                                                     L.ptr(lin.bias), lin.out_features,
                                                     lin.act if act is None else act, L.ptr(out),
                                                     out.stride(0), L.ptr(sbits),
                                                     0 if sbits is None else sbits.stride(0), L.stream_ptr()))
    return out


def _cell_step(netmon, cell, x_src, h_ptr, ldh, c_ptr, ldc, S, M, tag_kind):
    """One NetMon RNN cell on A = [x_src | h] writing the new state rows S ([h | c] for the
    LSTMs, h for GRU): lstm / gru one gate-tile GEMM with the gate math in its epilogue; lnlstm
    two GEMMs (x W_ih^T, h W_hh^T) + gm_lnlstm_pointwise (the LayerNorms need whole rows)."""
    H = netmon.hidden_features
    SW = S.stride(0)
    rnn = netmon.rnn_type
    ctag = getattr(cell, "tag", None)
    tag = ctag and f"{tag_kind}:{ctag}:{M}x{4 * H}x{2 * H}"
    if rnn == "lstm":
        wp, ldw, bp, x3 = pack_lstm(cell)
        gemm(x_src, dense(h_ptr, ldh, H), wp.data_ptr(), ldw, bp.data_ptr(), M, 4 * H, GM_EPI_LSTM, S.data_ptr(), SW,
             S.data_ptr() + 4 * H, SW, c_ptr, ldc, tag=tag, x3=x3)
    elif rnn == "gru":
        wp, ldw, bp, x3 = pack_gru(cell)
        gemm(x_src, dense(h_ptr, ldh, H), wp.data_ptr(), ldw, bp.data_ptr(), M, 4 * H, GM_EPI_GRU, S.data_ptr(), SW,
             c_in=h_ptr, ldc=ldh, tag=tag, x3=x3)
    elif rnn == "lnlstm":
        (wi, ldi, xi), (wh, ldhw, xh) = pack_lnlstm(cell)
        G = torch.empty(M, 8 * H, device=S.device)  # stream-ordered allocator: safe across stream groups
        with L.timed(tag):
            gemm(x_src, None, wi.data_ptr(), ldi, None, M, 4 * H, GM_EPI_BIAS, G.data_ptr(), 8 * H, x3=xi)
            gemm(dense(h_ptr, ldh, H), None, wh.data_ptr(), ldhw, None, M, 4 * H, GM_EPI_BIAS, G.data_ptr() + 16 * H,
                 8 * H, x3=xh)
            li, lh, lc = cell.ln_input, cell.ln_hidden, cell.ln_cell
            L.check(L.lib().gm_lnlstm_pointwise(G.data_ptr(), 8 * H, c_ptr, ldc, li.weight.data_ptr(), li.bias.data_ptr(),
                                                lh.weight.data_ptr(), lh.bias.data_ptr(), cell.bias_ih.data_ptr(),
                                                lc.weight.data_ptr(), lc.bias.data_ptr(), M, H, float(li.eps),
                                                S.data_ptr(), SW, S.data_ptr() + 4 * H, SW, L.stream_ptr()))
    else:
        raise NotImplementedError(f"fused NetMon step: rnn_type {rnn!r}")


def fused_ok(netmon):
    """The fused no-grad NetMon step covers lstm / lnlstm / gru with state carry-over and the
    neighbour readout (the reference's NetMonWrapper configuration on routing graphs)."""
    return (netmon.rnn_type in ("lstm", "lnlstm", "gru") and netmon.rnn_carryover and netmon.output_neighbor_hidden
            and not netmon.output_global_hidden and netmon.hidden_features % 32 == 0)


@torch.no_grad()
def netmon_step(netmon, node_obs, nbr, state, out=None, last_out=None):
    """One NetMon step for B graphs. node_obs [B, N, F]; nbr int32 [B, N, deg]; state
    [B, N, S] (S = 2H [h | c] for lstm / lnlstm, H for gru) or None. Returns (new state
    [B, N, S], h_prev rows [B*N, S] whose first H columns are the last pre-aggregation h).
    out / last_out ([B*N, S], optional) receive the new state and h_prev, so a caller can keep
    them in fixed buffers (graph replay)."""
    if not fused_ok(netmon):
        raise NotImplementedError("fused NetMon step: lstm / lnlstm / gru with carry-over (else NetMon.forward_graph)")
    B, N, Fd = node_obs.shape
    H = netmon.hidden_features
    SW = netmon.state_size
    M = B * N
    dev = node_obs.device
    x = node_obs.reshape(M, Fd)
    layers = list(netmon.encode.linear_layers)
    if encoder_chain_ok(layers, N, Fd, nbr):  # layers 1-3 in one launch (gm_encoder_x3)
        l0, l1, l2 = layers[:3]
        x = encoder_chain(l0, l1, l2, x, nbr, N, torch.empty(M, l2.out_features, device=dev))
        layers = layers[3:]
    elif renc_fold_ok(layers, N, Fd, nbr):  # layers 1 and 2 in one GEMM: layer 1 computed in layer 2's A load
        l0, l1 = layers[0], layers[1]
        y = torch.empty(M, l1.out_features, device=dev)
        gemm(routing_enc_src(l0, x, nbr, N), None, None, 0, l1.bias.data_ptr(), M, l1.out_features, _epi(l1.act),
             y.data_ptr(), y.stride(0), tag=l1.tag and f"linear:{l1.tag}:{M}x{l1.out_features}x{l1.in_features}",
             x3=pack_x3(l1))
        x = y
        layers = layers[2:]
    elif routing_encoder_ok(layers[0], N, Fd, nbr):
        x = routing_encoder(layers[0], x, nbr, B, N, torch.empty(M, layers[0].out_features, device=dev))
        layers = layers[1:]
    for lin in layers:
        x = _linear(x, x.stride(0), x.shape[1], lin, torch.empty(M, lin.out_features, device=dev))
    if state is None:
        state = torch.zeros(B, N, SW, device=dev)
    st = state.reshape(M, SW)
    K = netmon.iterations
    cstate = SW > H  # LSTMs carry c in the second half of the row

    def buf(i):  # storage of S_i (S_0 = obs cell output, S_K = new state, S_{K-1} = h_prev)
        if i == K and out is not None:
            return out.reshape(M, SW)
        if i == K - 1 and last_out is not None:
            return last_out.reshape(M, SW)
        return torch.empty(M, SW, device=dev)

    S = buf(0)
    _cell_step(netmon, netmon.rnn_obs, dense(x.data_ptr(), x.stride(0), H), st.data_ptr(), SW,
               st.data_ptr() + 4 * H if cstate else None, SW, S, M, "lstm")
    last = S
    mean = netmon.agg_mode == 1
    agg = torch.empty(M, H, device=dev) if PRE_AGG else None
    for it in range(K):
        last = S
        S2 = buf(it + 1)
        if PRE_AGG:  # aggregate pass, then the update cell on dense [Σ h | h]
            with L.timed(f"mp_aggregate:{M}x{H}"):
                L.check(L.lib().gm_mp_aggregate_rows(S.data_ptr(), SW, nbr.data_ptr(), B, N, nbr.shape[-1], H,
                                                     int(mean), agg.data_ptr(), H, L.stream_ptr()))
            a_src = dense(agg.data_ptr(), H, H)
        else:
            a_src = aggregate(S.data_ptr(), SW, H, nbr, N, mean)
        _cell_step(netmon, netmon.rnn_update, a_src, S.data_ptr(), SW, S.data_ptr() + 4 * H if cstate else None, SW,
                   S2, M, "lstm_agg")
        S = S2
    if K <= 0:
        last = torch.zeros_like(S)
    netmon.state = S.view(B, N, SW)
    return netmon.state, last


@torch.no_grad()
def dqn_q(dqn, env_obs, obs_dim, state, h_prev, nbr, agent_node, scratch, hidden=None, obs_gemm=None):
    """Q [B*A, actions] of the DQN on [env obs | NetMon readout] with the readout gathered
    inside the first GEMM. env_obs: [B, A, stride] (first obs_dim columns used); state rows
    [h | ...] of width state.shape[-1] (hidden H: default half the width, the LSTM layout).
    obs_gemm: the env's GEMM-ready copy [B, A, 6N+8] (Routing.enable_gemm_obs): read instead of
    env_obs with the folded weights (K two columns shorter: whole k tiles at N = 20)."""
    B, A, stride = env_obs.shape
    N = nbr.shape[1]
    H = hidden or state.shape[-1] // 2
    M = B * A
    lin0 = dqn.encoder.linear_layers[0]
    fold = obs_gemm is not None and obs_dim == 6 * N + 10
    wp, ldw, b, x3 = pack_dqn_first(lin0, obs_dim, N if fold else None)
    if fold:
        src, ks = dense(obs_gemm.data_ptr(), obs_gemm.stride(1), obs_dim - 2), obs_dim - 2
    else:
        src, ks = dense(env_obs.data_ptr(), stride, obs_dim), obs_dim
    a0 = readout(state.data_ptr(), state.shape[-1], h_prev.data_ptr(), h_prev.stride(0), nbr, agent_node, N, H)
    h1 = scratch(0, M, lin0.out_features)
    gemm(a0, src, wp.data_ptr(), ldw, b.data_ptr(), M, lin0.out_features,
         _epi(lin0.act), h1.data_ptr(), h1.stride(0),
         tag=lin0.tag and f"linear:{lin0.tag}:{M}x{lin0.out_features}x{a0.k + ks}", x3=x3)
    h = h1
    hidden = list(dqn.encoder.linear_layers[1:])
    fc = dqn.q_net.fc
    fuse = len(hidden) > 0 and head_ok(hidden[-1], fc)
    for i, lin in enumerate(hidden[:-1] if fuse else hidden + [fc]):
        h = _linear(h, h.stride(0), h.shape[1], lin, scratch(i + 1, M, lin.out_features))
    if fuse:  # last hidden layer + Q head in one kernel
        h = linear_head(hidden[-1], fc, h, h.stride(0), h.shape[1], scratch(len(hidden) + 1, M, fc.out_features))
    return h


@torch.no_grad()
def dqn_q_dense(dqn, env_obs, graph, scratch):
    """Q [B*A, actions] of the DQN on [env obs | graph obs] given as two dense sources (the training
    target pass on the online graph observations): env_obs [B, A, od] with 16-byte rows, graph
    [B, A, G] contiguous."""
    B, A, od = env_obs.shape
    M = B * A
    g2 = graph.reshape(M, graph.shape[-1])
    lin0 = dqn.encoder.linear_layers[0]
    wp, ldw, b, x3 = pack_dqn_first(lin0, od)
    h1 = scratch(0, M, lin0.out_features)
    gemm(dense(g2.data_ptr(), g2.stride(0), g2.shape[1]), dense(env_obs.data_ptr(), env_obs.stride(1), od),
         wp.data_ptr(), ldw, b.data_ptr(), M, lin0.out_features, _epi(lin0.act),
         h1.data_ptr(), h1.stride(0), tag=lin0.tag and f"linear:{lin0.tag}:{M}x{lin0.out_features}x{g2.shape[1]}+{od}",
         x3=x3)
    h = h1
    hidden = list(dqn.encoder.linear_layers[1:])
    fc = dqn.q_net.fc
    fuse = len(hidden) > 0 and head_ok(hidden[-1], fc)
    for i, lin in enumerate(hidden[:-1] if fuse else hidden + [fc]):
        h = _linear(h, h.stride(0), h.shape[1], lin, scratch(i + 1, M, lin.out_features))
    if fuse:
        h = linear_head(hidden[-1], fc, h, h.stride(0), h.shape[1], scratch(len(hidden) + 1, M, fc.out_features))
    return h
