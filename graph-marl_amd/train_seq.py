"""Sequence-batched DQN + NetMon update (reference src/main.py:840-1026 on replay sequences,
src/replaybuffer.py:103-130) with a hand-written backward.

The reference runs, per step t of a sampled sequence of L consecutive transitions, NetMon on
the stored node observations (state carried from the stored start state, reset at episode
ends), the DQN on [env obs | NetMon readout], the target DQN on the next observation, and
backpropagates the summed TD loss through all of it with autograd. Here the same computation
is one autograd node over the whole sequence (`_SeqFn`), organised for the GPU:

  * everything without recurrence runs ONCE over all L steps' rows: the NetMon encoder MLP
    (L*B*N rows), the readout, the DQN (L*B*A rows), their weight gradients, and the target
    DQN of steps 0..L-2 (whose next observations are the online ones of steps 1..L-1);
  * only the LSTM cells and the aggregate run per step (forward: one [x | h] GEMM per cell with
    the gate math in its epilogue; backward: gm_lstm_cell_bwd, which sums every gradient source
    of the cell — readout, the next cell's input gradient, the transposed aggregate, the next
    step's state gradient masked at episode ends — and one input-gradient GEMM per cell);
  * the leaky_relu derivative, the bias-gradient column sums and the gradient scales are fused
    into the kernels that produce the gradients (gm_gemm_x3_dgrad, gm_qhead_bwd,
    gm_lstm_cell_bwd), so no activation gradient is re-read for them.

Every GEMM runs in the split-f16 form with fp32 accumulation (gm_gemm_x3 / gm_gemm_x3_wgrad),
as in the autograd path (train.dqn_loss), which remains the path for every other configuration
(GRU / LN-LSTM cells, no carry-over, global readout, aux loss, DGN/DQNR/CommNet, GM_GEMM=f32).
"""
import ctypes as C
from collections import namedtuple

import torch

from . import _lib as L
from . import fused as FU
from . import model as MD

SeqBatch = namedtuple("SeqBatch", ["obs", "obs_dim", "action", "reward", "done", "episode_done", "node_obs", "nbr",
                                   "agent_node", "node_state", "next_fields", "idx"], defaults=(None,))
"""All L steps of B replay sequences, stacked: obs [L, B, A, odp] (rows padded to 16 bytes, first
obs_dim columns valid), action [L, B, A] long, reward [L, B, A], done [L, B, A] bool, episode_done
[L, B] bool, node_obs [L, B, N, F], nbr [L, B, N, deg] int32, agent_node [L, B, A] int32,
node_state [B, N, 2H] (the NetMon state before step 0). next_fields(t, rows) -> (next_obs
[len, A, odp], next_node_obs [len, N, F], next_agent_node [len, A] int32) of step t for the
sequences `rows` (None = all)."""


def seq_ok(netmon, model, model_tar, att_coeff=0.0, aux_model=None):
    """The sequence-batched path covers the reference's NetMon + DQN configuration: LSTM cells with
    carry-over, sum / mean aggregation, neighbour readout, leaky MLPs, split-f16 GEMMs."""
    if netmon is None or aux_model is not None or att_coeff != 0 or L.GEMM_MODE != "x3":
        return False
    if type(model) is not MD.DQN or type(model_tar) is not MD.DQN:
        return False
    H = netmon.hidden_features
    enc = list(netmon.encode.linear_layers)
    dq = list(model.encoder.linear_layers)
    fc = model.q_net.fc
    return (netmon.rnn_type == "lstm" and netmon.rnn_carryover and netmon.output_neighbor_hidden
            and not netmon.output_global_hidden and netmon.iterations >= 1 and H % 32 == 0 and H <= 1024
            and all(l.act == 1 for l in enc) and all(l.act == 1 for l in dq) and fc.act == 0
            and fc.out_features <= 4 and all(l.bias is not None for l in enc + dq + [fc])
            and dq[-1].out_features <= 1024)


def _zeros1(dev):
    return torch.zeros(1, device=dev)


def _finish(slot):
    L.check(FU._setup().gm_absmax_finish(slot.data_ptr(), L.stream_ptr()))
    return slot


class _X3Cache:
    """Split-f16 packs a module's training GEMMs need, refreshed when a parameter changes."""

    def __init__(self):
        self.p = {}

    def get(self, name, key, fn):
        k, v = self.p.get(name, (None, None))
        if k != key:
            v = fn()
            self.p[name] = (key, v)
        return v


def _cache(mod):
    if not hasattr(mod, "_seq_x3"):
        mod._seq_x3 = _X3Cache()
    return mod._seq_x3


def _x3(w):
    """X3 of an [n][k] weight (any n: the narrow tiles too)."""
    wp, ldw = FU._pad_cols(w.detach())
    return FU.X3(wp, ldw, w.shape[0], w.shape[1])


def _lin_x3(lin):
    return _cache(lin).get("fwd", FU._key(lin.weight), lambda: _x3(lin.weight))


def _lin_x3t(lin, cols=None):
    """X3 of W^T (or of W[:, cols]^T) for the input gradient gx = g @ W."""
    def build():
        w = lin.weight.detach() if cols is None else lin.weight.detach()[:, cols]
        return _x3(w.t().contiguous())
    return _cache(lin).get(("t", None if cols is None else (cols.start, cols.stop)), FU._key(lin.weight), build)


def _dqn_first_x3(lin, od):
    """First DQN layer with columns reordered to [graph | env obs] (the GEMM's two sources)."""
    def build():
        with torch.no_grad():
            w = torch.cat([lin.weight[:, od:], lin.weight[:, :od]], 1)
            return _x3(w)
    return _cache(lin).get(("first", od), FU._key(lin.weight), build)


def _lstm_x3t(cell):
    """X3 of [W_ih | W_hh]^T ([2H][4H], natural gate order) for d[x | h] = dgates @ [W_ih | W_hh]."""
    def build():
        w = torch.cat([cell.weight_ih.detach(), cell.weight_hh.detach()], 1)
        return _x3(w.t().contiguous())
    return _cache(cell).get("t", FU._key(cell.weight_ih, cell.weight_hh), build)


def _lstm_fwd(cell):
    """Interleaved gate-tile pack of the cell (fused.pack_lstm) with its split-f16 form forced."""
    wp, ldw, bp, x3 = FU.pack_lstm(cell)
    if x3 is None:
        x3 = _cache(cell).get("fwdx3", FU._key(cell.weight_ih, cell.weight_hh), lambda: FU.X3(wp, ldw, wp.shape[0],
                                                                                                2 * cell.hidden_size))
    return wp, ldw, bp, x3


def _ptr(t):
    return t if isinstance(t, int) else t.data_ptr()


def _sign_bits(rows, n, dev):
    """uint32 sign words of an activation (bit c % 32 of word c / 32: value > 0), int32 storage."""
    return torch.empty(rows, (n + 31) // 32, dtype=torch.int32, device=dev)


def _gemm_amax(x, ldx, k, x3, b, m, n, epi, y, ldy, slot, a1=None, sbits=None):
    """y = epi([x | a1] @ W^T + b) in split-f16 form, max |A| published into slot; a1 = (tensor, ld,
    k1) or None; sbits (optional) receives y's sign bits."""
    src1 = None if a1 is None else FU.dense(_ptr(a1[0]), a1[1], a1[2])
    FU.gemm(FU.dense(_ptr(x), ldx, k, amax=slot.data_ptr()), src1, None, 0, None if b is None else b.data_ptr(), m,
            n, epi, _ptr(y), ldy, ldc=0 if sbits is None else sbits.stride(0),
            act_out=None if sbits is None else sbits.data_ptr(), x3=x3)


def _dgrad(g, ldg, k, sc, x3t, m, n, split, mask, ldm, y, ldy, y2=None, ldy2=0, part=None, gmax=None):
    """gm_gemm_x3_dgrad (part rows = 128-row tiles); mask = the layer input's sign bits (int32 words,
    ldm words per row) or None."""
    a = FU.dense(_ptr(g), ldg, k, scale=sc.data_ptr())
    L.check(FU._setup().gm_gemm_x3_dgrad(C.byref(a), x3t.wp.data_ptr(), x3t.sinv.data_ptr(), m, n, split,
                                         None if mask is None else _ptr(mask), ldm, _ptr(y), ldy,
                                         None if y2 is None else _ptr(y2), ldy2, None if part is None else part.data_ptr(),
                                         None if gmax is None else gmax.data_ptr(), L.stream_ptr()))


class _Plan:
    """Inputs, modules and the forward's saved tensors of one sequence update."""
    pass


def _forward(p):
    netmon, dqn = p.netmon, p.dqn
    sb = p.seq
    dev = sb.obs.device
    Ls, B, A, odp = sb.obs.shape
    N, F = sb.node_obs.shape[2], sb.node_obs.shape[3]
    od = sb.obs_dim
    H = netmon.hidden_features
    S2 = 2 * H
    K = netmon.iterations
    M, Ma = B * N, B * A
    LM, LMa = Ls * M, Ls * Ma
    p.dims = (Ls, B, A, N, F, od, odp, H, K, M, Ma)
    mean = int(netmon.agg_mode == 1)
    X = sb.node_obs.reshape(LM, F)
    if X.stride(0) % 4 or X.data_ptr() % 16:
        Xp = torch.zeros(LM, (F + 3) // 4 * 4, device=dev)
        Xp[:, :F] = X
        X = Xp
    nbr = sb.nbr.reshape(Ls * B, N, -1).contiguous()
    an = sb.agent_node.reshape(Ls * B, A).contiguous()
    p.nbr, p.an = nbr, an
    deg = nbr.shape[-1]

    # ---- NetMon encoder over all steps ----
    enc = list(netmon.encode.linear_layers)
    p.enc_in, p.enc_out, p.enc_bits = [], [], []
    x, ldx, kx = X, X.stride(0), F
    for i, lin in enumerate(enc):
        n = lin.out_features
        y = torch.empty(LM, n, device=dev)
        yb = _sign_bits(LM, n, dev)  # the leaky mask of this output for the backward
        if i == 0 and FU.routing_encoder_ok(lin, N, F, nbr):
            FU.routing_encoder(lin, X, nbr, Ls * B, N, y, sbits=yb)
            sx = torch.empty(1, device=dev)
            L.check(FU._setup().gm_absmax_scale_rows(X.data_ptr(), LM, F, X.stride(0), sx.data_ptr(), L.stream_ptr()))
        else:
            sx = _zeros1(dev)
            _gemm_amax(x, ldx, kx, _lin_x3(lin), lin.bias, LM, n, FU.GM_EPI_BIAS_LEAKY, y, n, sx, sbits=yb)
            _finish(sx)
        p.enc_in.append((x, ldx, kx, sx))
        p.enc_out.append(y)
        p.enc_bits.append(yb)
        x, ldx, kx = y, n, n
    E = p.enc_out[-1]  # [LM][H], the obs cell's x

    # ---- LSTM cells, per step ----
    S_in = torch.empty(Ls, M, S2, device=dev)
    S = torch.empty(K + 1, Ls, M, S2, device=dev)  # cell outputs [h | c]: j = 0 obs, 1..K update
    act = torch.empty(K + 1, Ls, M, 4 * H, device=dev)
    agg = torch.empty(K, Ls, M, H, device=dev)
    s_obs, s_upd = _zeros1(dev), _zeros1(dev)
    wo = _lstm_fwd(netmon.rnn_obs)
    wu = _lstm_fwd(netmon.rnn_update)
    keep = (~sb.episode_done).to(torch.float32)  # [L, B]
    S_in[0].copy_(sb.node_state.reshape(M, S2))
    lib = L.lib()
    for t in range(Ls):
        if t > 0:  # the state carried from step t-1, zeroed at its episode end (src/main.py:858-866)
            torch.mul(S[K, t - 1].view(B, N * S2), keep[t - 1].view(B, 1), out=S_in[t].view(B, N * S2))
        src, sh = E[t * M:(t + 1) * M], S_in[t]
        for j in range(K + 1):
            wp, ldw, bp, x3 = wo if j == 0 else wu
            if j == 0:
                xa, hsrc = FU.dense(src.data_ptr(), H, H, amax=s_obs.data_ptr()), sh
            else:
                prev = S[j - 1, t]
                L.check(lib.gm_mp_aggregate_rows(prev.data_ptr(), S2, nbr[t * B:(t + 1) * B].data_ptr(), B, N, deg, H,
                                                 mean, agg[j - 1, t].data_ptr(), H, L.stream_ptr()))
                xa, hsrc = FU.dense(agg[j - 1, t].data_ptr(), H, H, amax=s_upd.data_ptr()), prev
            out = S[j, t]
            FU.gemm(xa, FU.dense(hsrc.data_ptr(), S2, H), wp.data_ptr(), ldw, bp.data_ptr(), M, 4 * H, FU.GM_EPI_LSTM,
                    out.data_ptr(), S2, out.data_ptr() + 4 * H, S2, hsrc.data_ptr() + 4 * H, S2, act[j, t].data_ptr(),
                    x3=x3)
    _finish(s_obs)
    _finish(s_upd)
    p.S_in, p.S, p.act, p.agg, p.s_obs, p.s_upd = S_in, S, act, agg, s_obs, s_upd

    # ---- readout + DQN over all steps ----
    R = torch.empty(LMa, 4 * H, device=dev)
    hp = S[K - 1] if K >= 1 else torch.zeros_like(S[K])
    L.check(lib.gm_netmon_readout_ld(S[K].data_ptr(), S2, hp.data_ptr(), S2, nbr.data_ptr(), an.data_ptr(), Ls * B, N,
                                     A, deg, H, R.data_ptr(), 4 * H, L.stream_ptr()))
    p.R = R
    env = sb.obs.reshape(LMa, odp)
    p.env = env
    dl = list(dqn.encoder.linear_layers)
    fc = dqn.q_net.fc
    nq = fc.out_features
    p.d, p.d_in_scale, p.d_bits = [], [], []
    q = torch.empty(LMa, nq, device=dev)
    for i, lin in enumerate(dl):
        n = lin.out_features
        y = torch.empty(LMa, n, device=dev)
        sx = _zeros1(dev)
        last = i == len(dl) - 1
        yb = None if last else _sign_bits(LMa, n, dev)
        p.d_bits.append(yb)
        if i == 0:
            _gemm_amax(R, 4 * H, 4 * H, _dqn_first_x3(lin, od), lin.bias, LMa, n, FU.GM_EPI_BIAS_LEAKY, y, n, sx,
                       a1=(env, odp, od), sbits=yb)
            if last:
                torch.addmm(fc.bias.detach(), y, fc.weight.detach().t(), out=q)
        elif last and n <= 256:  # last hidden layer + Q head in one kernel (hidden output written too)
            prev = p.d[-1]
            kp = prev.shape[1]
            x3 = _lin_x3(lin)
            wq = fc.weight.detach().contiguous()
            L.check(FU._setup().gm_gemm_x3_head(
                C.byref(FU.dense(prev.data_ptr(), kp, kp, amax=sx.data_ptr())), x3.wp.data_ptr(), x3.sinv.data_ptr(),
                lin.bias.data_ptr(), LMa, n, 1, wq.data_ptr(), wq.stride(0), fc.bias.data_ptr(), nq, q.data_ptr(), nq,
                y.data_ptr(), n, L.stream_ptr()))
        else:
            prev = p.d[-1]
            _gemm_amax(prev, prev.shape[1], prev.shape[1], _lin_x3(lin), lin.bias, LMa, n, FU.GM_EPI_BIAS_LEAKY, y, n,
                       sx, sbits=yb)
            if last:
                torch.addmm(fc.bias.detach(), y, fc.weight.detach().t(), out=q)
        p.d.append(y)
        p.d_in_scale.append(_finish(sx))
    return q


def _wgrad(g, sa, x, k, sb_):
    """dW = g^T x[:, :k] (split-K split-f16 kernel; both operand scales given)."""
    return MD._wgrad(g, x, k, sa, sb_)


def _backward(p, dq):
    netmon, dqn = p.netmon, p.dqn
    Ls, B, A, N, F, od, odp, H, K, M, Ma = p.dims
    S2 = 2 * H
    dev = dq.device
    LM, LMa = Ls * M, Ls * Ma
    lib = L.lib()
    grads = {}
    dq = dq.contiguous()

    # ---- DQN ----
    dl = list(dqn.encoder.linear_layers)
    fc = dqn.q_net.fc
    nq = fc.out_features
    nl = len(dl)
    dlast = p.d[-1]
    n_last = dlast.shape[1]
    rpb = 512
    nb = (LMa + rpb - 1) // rpb
    g = torch.empty(LMa, n_last, device=dev)
    part_b = torch.empty(nb, n_last, device=dev)
    part_wq = torch.empty(nb, nq, n_last, device=dev)
    part_bq = torch.empty(nb, nq, device=dev)
    sc = torch.empty(1, device=dev)
    wq = fc.weight.detach().contiguous()
    L.check(lib.gm_qhead_bwd(dq.data_ptr(), nq, nq, wq.data_ptr(), wq.stride(0), dlast.data_ptr(), n_last, LMa, n_last,
                             1, g.data_ptr(), n_last, part_b.data_ptr(), part_wq.data_ptr(), part_bq.data_ptr(), rpb,
                             sc.data_ptr(), L.stream_ptr()))
    grads[fc.weight] = part_wq.sum(0)
    grads[fc.bias] = part_bq.sum(0)
    grads[dl[-1].bias] = part_b.sum(0)
    for i in range(nl - 1, 0, -1):
        lin = dl[i]
        xin = p.d[i - 1]
        kin = xin.shape[1]
        grads[lin.weight] = _wgrad(g, sc, xin, kin, p.d_in_scale[i])
        gn = torch.empty(LMa, kin, device=dev)
        part = torch.empty((LMa + 127) // 128, kin, device=dev)
        gmax = _zeros1(dev)
        xb = p.d_bits[i - 1]
        _dgrad(g, lin.out_features, lin.out_features, sc, _lin_x3t(lin), LMa, kin, kin, xb, xb.stride(0), gn, kin,
               part=part, gmax=gmax)
        grads[dl[i - 1].bias] = part.sum(0)
        g, sc = gn, _finish(gmax)
    lin0 = dl[0]
    s_in0 = p.d_in_scale[0]
    w_r, w_env = MD._wgrad_pair(g, p.R, 4 * H, p.env, od, sc, s_in0, s_in0)  # one launch: g read once per k chunk
    grads[lin0.weight] = torch.cat([w_env, w_r], 1)
    dR = torch.empty(LMa, 4 * H, device=dev)
    _dgrad(g, lin0.out_features, lin0.out_features, sc, _lin_x3t(lin0, slice(od, od + 4 * H)), LMa, 4 * H, 4 * H,
           None, 0, dR, 4 * H)

    # ---- readout over all steps ----
    dhf = torch.empty(LM, H, device=dev)
    dhp = torch.empty(LM, H, device=dev)
    L.check(lib.gm_netmon_readout_bwd(dR.data_ptr(), 4 * H, p.nbr.data_ptr(), p.an.data_ptr(), Ls * B, N, A,
                                      p.nbr.shape[-1], H, dhf.data_ptr(), dhp.data_ptr(), L.stream_ptr()))

    # ---- LSTM cells, per step, in reverse ----
    dG = torch.empty(K + 1, Ls, M, 4 * H, device=dev)
    rpb_c = 64
    nbc = (M + rpb_c - 1) // rpb_c
    bpart = torch.empty(K + 1, Ls, nbc, 4 * H, device=dev)
    gmax_obs, gmax_upd = _zeros1(dev), _zeros1(dev)
    E = p.enc_out[-1]
    gE = torch.empty(LM, H, device=dev)
    nbe = (M + 127) // 128
    partE = torch.empty(Ls, nbe, H, device=dev)
    gmaxE = _zeros1(dev)
    wt_obs, wt_upd = _lstm_x3t(netmon.rnn_obs), _lstm_x3t(netmon.rnn_update)
    ep_done = p.seq.episode_done.to(torch.uint8).contiguous()  # [L, B]
    dh_ext = dc_ext = None
    sc_cell = torch.empty(1, device=dev)
    D = torch.empty(M, S2, device=dev)
    dh0_buf = [torch.empty(M, H, device=dev), torch.empty(M, H, device=dev)]
    # every cell's dc source is the dc output of the cell processed just before it (the next cell
    # of the step, or step t+1's obs cell): two buffers in turn
    dc_buf = [torch.empty(M, H, device=dev), torch.empty(M, H, device=dev)]
    calls = 0
    mean = int(netmon.agg_mode == 1)
    deg = p.nbr.shape[-1]
    for t in range(Ls - 1, -1, -1):
        nbr_t = p.nbr[t * B:(t + 1) * B]
        dc_next = None
        have_D = False
        for j in range(K, -1, -1):
            a = L.LSTMBwdArgs()
            a.act, a.ld_act = p.act[j, t].data_ptr(), 4 * H
            cin = p.S_in[t] if j == 0 else p.S[j - 1, t]
            a.c_in, a.ld_cin = cin.data_ptr() + 4 * H, S2
            a.c_out, a.ld_cout = p.S[j, t].data_ptr() + 4 * H, S2
            if j == K:
                a.dh0, a.ld_dh0 = dhf[t * M:(t + 1) * M].data_ptr(), H
            else:
                a.dh0, a.ld_dh0 = D.data_ptr() + 4 * H, S2  # h part of the next cell's input gradient
                a.dm, a.ld_dm = D.data_ptr(), S2            # its aggregate part, transposed
                a.nbr, a.n_nodes, a.deg, a.mean = nbr_t.data_ptr(), N, deg, mean
            if j == K - 1:
                a.dh1, a.ld_dh1 = dhp[t * M:(t + 1) * M].data_ptr(), H
            if j == K and dh_ext is not None:  # step t+1's input-state gradient, zero where episode t ended
                a.dh_ext, a.ld_ext = dh_ext.data_ptr(), H
                a.dc_ext, a.ld_dcext = dc_ext.data_ptr(), H
                a.ext_mask, a.rows_per_sample = ep_done[t].data_ptr(), N
            if dc_next is not None:
                a.dc, a.ld_dc = dc_next.data_ptr(), H
            a.m, a.hidden = M, H
            a.dgates, a.ld_dg = dG[j, t].data_ptr(), 4 * H
            dco = None
            if j > 0 or t > 0:  # the gradient w.r.t. the replayed start state is not needed
                dco = dc_buf[calls % 2]
                a.dc_out, a.ld_dco = dco.data_ptr(), H
            calls += 1
            a.bias_part, a.rows_per_block = bpart[j, t].data_ptr(), rpb_c
            a.dg_scale = sc_cell.data_ptr()
            a.dg_max = (gmax_obs if j == 0 else gmax_upd).data_ptr()
            L.check(lib.gm_lstm_cell_bwd(C.byref(a), L.stream_ptr()))
            if j > 0:
                _dgrad(dG[j, t], 4 * H, 4 * H, sc_cell, wt_upd, M, S2, S2, None, 0, D, S2)
            else:
                # [x | h] input gradient of the obs cell: x part through the encoder's last leaky_relu
                # (bias partials and max for the batched encoder backward), h part = the state gradient
                dh0 = dh0_buf[t % 2]
                Eb = p.enc_bits[-1]
                _dgrad(dG[0, t], 4 * H, 4 * H, sc_cell, wt_obs, M, S2, H, Eb[t * M:(t + 1) * M], Eb.stride(0),
                       gE[t * M:(t + 1) * M], H, dh0, H, part=partE[t], gmax=gmaxE)
                dh_ext, dc_ext = dh0, dco
            dc_next = dco
    # LSTM weight / bias gradients over all steps (and update iterations)
    for j0, cell, gm_, sx, xs, hs in ((0, netmon.rnn_obs, gmax_obs, p.s_obs, E, p.S_in.reshape(LM, S2)),
                                      (1, netmon.rnn_update, gmax_upd, p.s_upd, p.agg.reshape(K * LM, H),
                                       p.S[:K].reshape(K * LM, S2))):
        gs = dG[j0:j0 + (1 if j0 == 0 else K)].reshape(-1, 4 * H)
        sa = _finish(gm_)
        grads[cell.weight_ih], grads[cell.weight_hh] = MD._wgrad_pair(gs, xs, H, hs, H, sa, sx, sx)
        bg = bpart[j0:j0 + (1 if j0 == 0 else K)].reshape(-1, 4 * H).sum(0)
        grads[cell.bias_ih] = bg
        grads[cell.bias_hh] = bg.clone()

    # ---- NetMon encoder over all steps ----
    enc = list(netmon.encode.linear_layers)
    g, sc = gE, _finish(gmaxE)
    grads[enc[-1].bias] = partE.reshape(-1, H).sum(0)
    for i in range(len(enc) - 1, -1, -1):
        lin = enc[i]
        xin, ldx, kin, sx = p.enc_in[i]
        grads[lin.weight] = _wgrad(g, sc, xin, kin, sx)
        if i > 0:
            gn = torch.empty(LM, kin, device=dev)
            part = torch.empty((LM + 127) // 128, kin, device=dev)
            gmax = _zeros1(dev)
            xb = p.enc_bits[i - 1]
            _dgrad(g, lin.out_features, lin.out_features, sc, _lin_x3t(lin), LM, kin, kin, xb, xb.stride(0), gn, kin,
                   part=part, gmax=gmax)
            grads[enc[i - 1].bias] = part.sum(0)
            g, sc = gn, _finish(gmax)
    return grads


class _SeqFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, *params):
        ctx.plan = plan
        with torch.no_grad():
            return _forward(plan)

    @staticmethod
    def backward(ctx, dq):
        p = ctx.plan
        grads = _backward(p, dq)
        ctx.plan = None
        return (None,) + tuple(grads.get(w) for w in p.params)


@torch.no_grad()
def _target_max(p, model_tar, gamma_unused=None):
    """max_a Q_target(next obs) [L, B, A]: steps 0..L-2 on the online observations of steps 1..L-1
    (one batched no-grad DQN pass; the target NetMon is the online NetMon, so its step t+1 is the
    online step t+1), except the sequences whose episode ended at t, which get their own NetMon
    step on the stored next observation; the last step runs its own NetMon step for all
    (src/main.py:878-915)."""
    from .train import _fused_next_q

    Ls, B, A, N, F, od, odp, H, K, M, Ma = p.dims
    sb = p.seq
    netmon = p.netmon
    dev = p.R.device
    out = torch.empty(Ls, B, A, device=dev)
    if Ls > 1:
        env = sb.obs[1:].reshape((Ls - 1) * B, A, odp)[..., :od]
        graph = p.R[Ma:].view((Ls - 1) * B, A, 4 * H)
        q = FU.dqn_q_dense(model_tar, env, graph, lambda i, m, n: torch.empty(m, n, device=dev))
        out[:-1] = q.view(Ls - 1, B, A, -1).max(dim=-1)[0]
        done_rows = sb.episode_done[:-1].nonzero().cpu()  # one host read per update
        for t in torch.unique(done_rows[:, 0]).tolist():
            r = done_rows[done_rows[:, 0] == t, 1].to(dev)
            no, nno, nan_ = sb.next_fields(t, r)
            st = p.S[K, t].view(B, N, 2 * H)[r]
            nb = sb.nbr[t][r]
            out[t, r] = _fused_next_q(netmon, model_tar, no[..., :od], nno, nb, nan_, st).max(dim=2)[0]
    no, nno, nan_ = sb.next_fields(Ls - 1, None)
    out[-1] = _fused_next_q(netmon, model_tar, no[..., :od], nno, sb.nbr[-1], nan_,
                            p.S[K, Ls - 1].view(B, N, 2 * H)).max(dim=2)[0]
    return out


def seq_loss(netmon, model, model_tar, seq, gamma, params, parts=None):
    """TD loss of src/main.py:840-1000 over a SeqBatch: (loss, q [L, B, A, nq], q_target)."""
    p = _Plan()
    p.netmon, p.dqn, p.seq, p.params = netmon, model, seq, list(params)
    q = _SeqFn.apply(p, *p.params)
    Ls, B, A = seq.action.shape
    q = q.view(Ls, B, A, -1)
    nxt = _target_max(p, model_tar)
    target = seq.reward + (~seq.done) * gamma * nxt
    q_target = torch.scatter(q.detach(), -1, seq.action.unsqueeze(-1), target.unsqueeze(-1))
    loss = (q - q_target).pow(2).mean(dim=(1, 2, 3)).sum() / Ls
    if parts is not None:
        parts.update(loss_q=loss, loss_att=None, loss_aux=None)
    return loss, q, q_target


def dqn_update_seq(netmon, model, model_tar, optimizer, params, seq, gamma, tau, target_update_steps=0, iteration=1,
                   group=None):
    """One update (src/main.py:840-1026) on a SeqBatch: the sequence-batched loss and backward, the
    gradient all-reduce across ranks, clip by value (0.5) and norm (1.0), AdamW, target update."""
    from .train import allreduce_gradients, interpolate_model

    loss, q, qt = seq_loss(netmon, model, model_tar, seq, gamma, params)
    optimizer.zero_grad(set_to_none=False)
    loss.backward()
    allreduce_gradients(params, group)
    torch.nn.utils.clip_grad_value_(params, 0.5)
    torch.nn.utils.clip_grad_norm_(params, 1.0)
    optimizer.step()
    if target_update_steps <= 0:
        interpolate_model(model, model_tar, tau, model_tar)
    elif iteration % target_update_steps == 0:
        model_tar.load_state_dict(model.state_dict())
    L.check_range()
    return loss.detach(), q, qt
