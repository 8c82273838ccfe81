"""Sequence-batched NetMon for the supervised driver (BASELINE config 5, reference src/sl.py:360-424)
with a hand-written backward.

The reference unrolls NetMon `sequence_length` times on the same graphs from a zero state
(src/sl.py:363-368), reads out every node after each step (NetMon without agent mapping,
src/sl.py:132-168, src/model.py:451-631) and backpropagates the mean of the per-step losses through
all of it with autograd. Here the NetMon part of the whole unroll is one autograd node (`_Fn`): its
output is the readout of every node at every step, [L, B*N, 4H]; the heads and the loss stay in
autograd and run once over all L steps' rows (sl.NetMonSL.forward_seq).

Forward: the encoder MLP once (the observations are the same at every step), then per step the obs
LSTM cell ([encoder output | h] as the GEMM's two sources, gate math in the epilogue) and K x
(aggregate, update cell), the state carried in place (S[K, t-1] is step t's input state), the
readout of every step.

Backward (the sequence-batched update's kernels, train_seq.py): the readout backward of every step,
then per step and cell, in reverse, gm_lstm_cell_bwd (sums the readout gradient, the next cell's h
gradient, the transposed aggregate of its x gradient and the next step's state gradient; writes the
gate gradients, bias partials and their scale) and one input-gradient GEMM per cell; the weight
gradients of the update cell over all steps at once; the encoder's gradient summed over the steps
(its output fed every step) before ONE encoder backward. No autograd accumulation of the h / c / encoder
gradients (the reference's graph adds them tensor by tensor).
"""
import ctypes as C

import torch

from . import _lib as L
from . import fused as FU
from . import train_seq as TS


def seq_bytes(netmon, rows, steps):
    """Device bytes the unroll keeps for its backward at M = rows node rows and L = steps: per cell and
    step the [h | c] output (2H), the gate activations (4H) and their gradient (4H), plus the K
    aggregates (H), all fp32."""
    H, K = netmon.hidden_features, netmon.iterations
    return 4 * steps * rows * ((K + 1) * 10 * H + K * H)


def _device_room(dev):
    free, _ = torch.cuda.mem_get_info(dev)
    return free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)


def seq_ok(netmon, rows=None, steps=None):
    """The configurations this path covers: LSTM cells with carry-over, sum / mean aggregation,
    neighbour readout without the global mean, leaky encoder layers with biases, split-f16 GEMMs;
    with rows / steps given, also that the unroll's saved tensors (seq_bytes) fit the device with a
    margin (otherwise the caller runs the per-step autograd path instead of failing with OOM)."""
    if netmon is None or L.GEMM_MODE != "x3":
        return False
    enc = list(netmon.encode.linear_layers)
    H = netmon.hidden_features
    ok = (netmon.rnn_type == "lstm" and netmon.rnn_carryover and netmon.output_neighbor_hidden
          and not netmon.output_global_hidden and netmon.iterations >= 1 and H % 32 == 0 and H <= 1024
          and len(enc) >= 1 and all(l.act == 1 and l.bias is not None for l in enc))
    if ok and rows is not None and steps is not None:
        # decided once per (module, rows, steps) shape: the allocator's free memory moves from step to
        # step, and the path (and with it the summation order) must not flip mid-run
        key = (rows, steps)
        cache = netmon.__dict__.setdefault("_sl_seq_fits", {})
        if key not in cache:
            dev = next(netmon.parameters()).device
            cache[key] = 1.25 * seq_bytes(netmon, rows, steps) < _device_room(dev)
        ok = cache[key]
    return ok


class _Plan:
    pass


def _forward(p):
    netmon = p.netmon
    X3d, nbr, Ls = p.x, p.nbr, p.steps
    dev = X3d.device
    B, N, F = X3d.shape
    H = netmon.hidden_features
    S2 = 2 * H
    K = netmon.iterations
    M = B * N
    p.dims = (Ls, B, N, F, H, K, M)
    mean = int(netmon.agg_mode == 1)
    X = X3d.reshape(M, F)
    if X.stride(0) % 4 or X.data_ptr() % 16:
        Xp = torch.zeros(M, (F + 3) // 4 * 4, device=dev)
        Xp[:, :F] = X
        X = Xp
    deg = nbr.shape[-1]
    lib = L.lib()

    # ---- encoder, once ----
    enc = list(netmon.encode.linear_layers)
    p.enc_in, p.enc_out, p.enc_bits = [], [], []
    x, ldx, kx = X, X.stride(0), F
    for i, lin in enumerate(enc):
        n = lin.out_features
        y = torch.empty(M, n, device=dev)
        yb = TS._sign_bits(M, n, dev)
        if i == 0 and FU.routing_encoder_ok(lin, N, F, nbr):
            FU.routing_encoder(lin, X, nbr, B, N, y, sbits=yb)
            sx = torch.empty(1, device=dev)
            L.check(FU._setup().gm_absmax_scale_rows(X.data_ptr(), M, F, X.stride(0), sx.data_ptr(), L.stream_ptr()))
        else:
            sx = TS._zeros1(dev)
            TS._gemm_amax(x, ldx, kx, TS._lin_x3(lin), lin.bias, M, n, FU.GM_EPI_BIAS_LEAKY, y, n, sx, sbits=yb)
            TS._finish(sx)
        p.enc_in.append((x, ldx, kx, sx))
        p.enc_out.append(y)
        p.enc_bits.append(yb)
        x, ldx, kx = y, n, n
    E = p.enc_out[-1]  # [M][H], every step's obs-cell input

    # ---- LSTM cells, per step; the state starts at zero (src/sl.py:365) ----
    S = torch.empty(K + 1, Ls, M, S2, device=dev)  # cell outputs [h | c]: j = 0 obs, 1..K update
    act = torch.empty(K + 1, Ls, M, 4 * H, device=dev)
    agg = torch.empty(K, Ls, M, H, device=dev)
    Z = torch.zeros(M, S2, device=dev)
    s_obs, s_upd = TS._zeros1(dev), TS._zeros1(dev)
    wo = TS._lstm_fwd(netmon.rnn_obs)
    wu = TS._lstm_fwd(netmon.rnn_update)
    for t in range(Ls):
        sh = Z if t == 0 else S[K, t - 1]
        for j in range(K + 1):
            wp, ldw, bp, x3 = wo if j == 0 else wu
            if j == 0:
                xa, hsrc = FU.dense(E.data_ptr(), H, H, amax=s_obs.data_ptr()), sh
            else:
                prev = S[j - 1, t]
                L.check(lib.gm_mp_aggregate_rows(prev.data_ptr(), S2, nbr.data_ptr(), B, N, deg, H, mean,
                                                 agg[j - 1, t].data_ptr(), H, L.stream_ptr()))
                xa, hsrc = FU.dense(agg[j - 1, t].data_ptr(), H, H, amax=s_upd.data_ptr()), prev
            out = S[j, t]
            FU.gemm(xa, FU.dense(hsrc.data_ptr(), S2, H), wp.data_ptr(), ldw, bp.data_ptr(), M, 4 * H, FU.GM_EPI_LSTM,
                    out.data_ptr(), S2, out.data_ptr() + 4 * H, S2, hsrc.data_ptr() + 4 * H, S2, act[j, t].data_ptr(),
                    x3=x3)
    TS._finish(s_obs)
    TS._finish(s_upd)
    p.S, p.act, p.agg, p.Z, p.s_obs, p.s_upd = S, act, agg, Z, s_obs, s_upd

    # ---- readout of every node at every step: [h_final | h before the last update of 3 neighbours] ----
    R = torch.empty(Ls * M, 4 * H, device=dev)
    for t in range(Ls):
        L.check(lib.gm_netmon_readout_ld(S[K, t].data_ptr(), S2, S[K - 1, t].data_ptr(), S2, nbr.data_ptr(), None, B,
                                         N, N, deg, H, R[t * M:(t + 1) * M].data_ptr(), 4 * H, L.stream_ptr()))
    netmon.set_state_hc(S[K, Ls - 1, :, :H], S[K, Ls - 1, :, H:], B, N)  # the state after the last step
    return R.view(Ls, M, 4 * H)


def _backward(p, dR):
    netmon = p.netmon
    Ls, B, N, F, H, K, M = p.dims
    S2 = 2 * H
    dev = dR.device
    nbr = p.nbr
    deg = nbr.shape[-1]
    lib = L.lib()
    grads = {}
    dR = dR.reshape(Ls * M, 4 * H).contiguous()

    # ---- readout, every step: dh_final of node v is row v's first segment of dR (read in place by the
    # cell backward, ld 4H); dh_prev gathered from the neighbours' segments (gm_netmon_readout_bwd, no agent map)
    dhp = torch.empty(Ls * M, H, device=dev)
    for t in range(Ls):
        L.check(lib.gm_netmon_readout_bwd(dR[t * M:(t + 1) * M].data_ptr(), 4 * H, nbr.data_ptr(), None, B, N, N, deg,
                                          H, None, dhp[t * M:(t + 1) * M].data_ptr(), L.stream_ptr()))

    # ---- LSTM cells, per step, in reverse ----
    S, act, Z = p.S, p.act, p.Z
    dG = torch.empty(K + 1, Ls, M, 4 * H, device=dev)
    rpb_c = 64
    nbc = (M + rpb_c - 1) // rpb_c
    bpart = torch.empty(K + 1, Ls, nbc, 4 * H, device=dev)
    gmax_obs, gmax_upd = TS._zeros1(dev), TS._zeros1(dev)
    gEs = torch.empty(Ls, M, H, device=dev)  # the encoder output's gradient from each step's obs cell
    nbe = (M + 127) // 128
    partE = torch.empty(Ls, nbe, H, device=dev)
    wt_obs, wt_upd = TS._lstm_x3t(netmon.rnn_obs), TS._lstm_x3t(netmon.rnn_update)
    sc_cell = torch.empty(1, device=dev)
    D = torch.empty(M, S2, device=dev)
    dh0_buf = [torch.empty(M, H, device=dev), torch.empty(M, H, device=dev)]
    dc_buf = [torch.empty(M, H, device=dev), torch.empty(M, H, device=dev)]
    Eb = p.enc_bits[-1]
    mean = int(netmon.agg_mode == 1)
    dh_ext = dc_ext = None
    calls = 0
    for t in range(Ls - 1, -1, -1):
        dc_next = None
        for j in range(K, -1, -1):
            a = L.LSTMBwdArgs()
            a.act, a.ld_act = act[j, t].data_ptr(), 4 * H
            cin = (Z if t == 0 else S[K, t - 1]) if j == 0 else S[j - 1, t]
            a.c_in, a.ld_cin = cin.data_ptr() + 4 * H, S2
            a.c_out, a.ld_cout = S[j, t].data_ptr() + 4 * H, S2
            if j == K:
                a.dh0, a.ld_dh0 = dR[t * M:(t + 1) * M].data_ptr(), 4 * H  # dh_final: segment 0 of dR
            else:
                a.dh0, a.ld_dh0 = D.data_ptr() + 4 * H, S2  # h part of the next cell's input gradient
                a.dm, a.ld_dm = D.data_ptr(), S2            # its aggregate part, transposed
                a.nbr, a.n_nodes, a.deg, a.mean = nbr.data_ptr(), N, deg, mean
            if j == K - 1:
                a.dh1, a.ld_dh1 = dhp[t * M:(t + 1) * M].data_ptr(), H
            if j == K and dh_ext is not None:  # step t+1's input-state gradient (no episode ends here)
                a.dh_ext, a.ld_ext = dh_ext.data_ptr(), H
                a.dc_ext, a.ld_dcext = dc_ext.data_ptr(), H
            if dc_next is not None:
                a.dc, a.ld_dc = dc_next.data_ptr(), H
            a.m, a.hidden = M, H
            a.dgates, a.ld_dg = dG[j, t].data_ptr(), 4 * H
            dco = None
            if j > 0 or t > 0:  # the gradient w.r.t. the zero start state is not needed
                dco = dc_buf[calls % 2]
                a.dc_out, a.ld_dco = dco.data_ptr(), H
            calls += 1
            a.bias_part, a.rows_per_block = bpart[j, t].data_ptr(), rpb_c
            a.dg_scale = sc_cell.data_ptr()
            a.dg_max = (gmax_obs if j == 0 else gmax_upd).data_ptr()
            L.check(lib.gm_lstm_cell_bwd(C.byref(a), L.stream_ptr()))
            if j > 0:
                TS._dgrad(dG[j, t], 4 * H, 4 * H, sc_cell, wt_upd, M, S2, S2, None, 0, D, S2)
            else:
                # [x | h] input gradient of the obs cell: x part through the encoder's last leaky_relu
                # (bias partials per step), h part = the state gradient of step t - 1
                dh0 = dh0_buf[t % 2]
                TS._dgrad(dG[0, t], 4 * H, 4 * H, sc_cell, wt_obs, M, S2, H, Eb, Eb.stride(0), gEs[t], H, dh0, H,
                          part=partE[t])
                dh_ext, dc_ext = dh0, dco
            dc_next = dco

    # ---- LSTM weight / bias gradients ----
    sa_obs, sa_upd = TS._finish(gmax_obs), TS._finish(gmax_upd)
    E = p.enc_out[-1]
    cell = netmon.rnn_obs
    # W_ih: every step's x is the same encoder output E: ONE launch over all L steps' gate gradients with E's
    # rows repeated (row map period M), instead of L launches of M rows (each at ~0.35 of the large-batch rate)
    r = TS.MD._wgrad2(dG[0].reshape(Ls * M, 4 * H), [(E, H, p.s_obs, M, 0)], sa_obs) if Ls > 1 else None
    if r is not None:
        grads[cell.weight_ih] = r[0]
    else:
        gw = None
        for t in range(Ls):
            w_t = TS._wgrad(dG[0, t], sa_obs, E, H, p.s_obs)
            gw = w_t if gw is None else gw.add_(w_t)
        grads[cell.weight_ih] = gw
    # W_hh: step 0's h is zero; step t's is S[K, t-1] (contiguous over t = 1..L-1)
    if Ls > 1:
        grads[cell.weight_hh] = TS._wgrad(dG[0, 1:].reshape(-1, 4 * H), sa_obs, S[K, :Ls - 1].reshape(-1, S2), H,
                                          p.s_obs)
    else:
        grads[cell.weight_hh] = torch.zeros_like(cell.weight_hh)
    bg = bpart[0].reshape(-1, 4 * H).sum(0)
    grads[cell.bias_ih] = bg
    grads[cell.bias_hh] = bg.clone()
    cell = netmon.rnn_update
    gs = dG[1:].reshape(-1, 4 * H)
    grads[cell.weight_ih], grads[cell.weight_hh] = TS.MD._wgrad_pair(gs, p.agg.reshape(K * Ls * M, H), H,
                                                                  S[:K].reshape(K * Ls * M, S2), H, sa_upd, p.s_upd,
                                                                  p.s_upd)
    bg = bpart[1:].reshape(-1, 4 * H).sum(0)
    grads[cell.bias_ih] = bg
    grads[cell.bias_hh] = bg.clone()

    # ---- encoder, once, on the gradient summed over the steps ----
    enc = list(netmon.encode.linear_layers)
    g = gEs.sum(0) if Ls > 1 else gEs[0]
    sc = torch.empty(1, device=dev)
    L.check(FU._setup().gm_absmax_scale(g.data_ptr(), g.numel(), sc.data_ptr(), L.stream_ptr()))
    grads[enc[-1].bias] = partE.reshape(-1, H).sum(0)
    for i in range(len(enc) - 1, -1, -1):
        lin = enc[i]
        xin, ldx, kin, sx = p.enc_in[i]
        grads[lin.weight] = TS._wgrad(g, sc, xin, kin, sx)
        if i > 0:
            gn = torch.empty(M, kin, device=dev)
            part = torch.empty((M + 127) // 128, kin, device=dev)
            gmax = TS._zeros1(dev)
            xb = p.enc_bits[i - 1]
            TS._dgrad(g, lin.out_features, lin.out_features, sc, TS._lin_x3t(lin), M, kin, kin, xb, xb.stride(0), gn,
                      kin, part=part, gmax=gmax)
            grads[enc[i - 1].bias] = part.sum(0)
            g, sc = gn, TS._finish(gmax)
    return grads


class _Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, *params):
        ctx.plan = plan
        with torch.no_grad():
            return _forward(plan)

    @staticmethod
    def backward(ctx, dR):
        p = ctx.plan
        grads = _backward(p, dR)
        ctx.plan = None
        return (None,) + tuple(grads.get(w) for w in p.params)


def readout_seq(netmon, x, nbr, steps):
    """NetMon unrolled `steps` times from a zero state on node observations x [B, N, F] with
    neighbour table nbr [B, N, deg] (int32): the readout of every node after every step,
    [steps, B*N, 4H], differentiable w.r.t. the NetMon parameters."""
    p = _Plan()
    p.netmon, p.x, p.nbr, p.steps = netmon, x, nbr.contiguous(), steps
    p.params = [w for w in netmon.parameters()]
    return _Fn.apply(p, *p.params)
