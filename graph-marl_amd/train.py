"""DQN + NetMon update on the device (reference src/main.py:819-1026) and the
data-parallel gradient exchange across GPUs.

Models: DQN, DGN (+ attention regularisation), DQNR, CommNet (agent state carried over
the sequence). Per update: for each step of the sampled sequence, NetMon re-runs with gradient
from the stored input state (reset on episode boundaries), its readout replaces
the graph part of the observation, the online DQN gives Q, the target DQN (online
NetMon, no grad) gives max Q of the next observation, the TD target is written
into the chosen action only (loss over all 4 actions, unchosen terms 0), loss
averaged over the sequence; then clip_grad_value(0.5), clip_grad_norm(1.0),
AdamW, soft target update. With world_size > 1 the gradients of all parameters
are averaged in ONE flattened RCCL all-reduce before clipping, so every rank
clips and steps on the global gradient and the replicas stay identical.
"""
import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import _lib as GL


class PeerFailure(RuntimeError):
    """A rank of the data-parallel job failed (raised on EVERY rank by the next gradient exchange or
    the end-of-training sync, so the ranks leave the training loop together)."""


def _distributed(group=None):
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


_BUCKET = {}


def _bucket(params):
    """The exchange's persistent buffers for this parameter list (no per-update allocation):
    the flat bucket (every parameter + the failure flag), a zero tensor per parameter for ranks / parameters
    without .grad, and the two flag values [0.], [1.]."""
    key = tuple((id(p), p.numel()) for p in params)
    b = _BUCKET.get(key)
    if b is None:
        p0 = params[0]
        n = sum(p.numel() for p in params) + 1
        b = (torch.empty(n, dtype=p0.dtype, device=p0.device), [torch.zeros_like(p) for p in params],
             (torch.zeros(1, dtype=p0.dtype, device=p0.device), torch.ones(1, dtype=p0.dtype, device=p0.device)))
        _BUCKET.clear()
        _BUCKET[key] = b
    return b


def allreduce_gradients(params, group=None, failed=False):
    """Average .grad over the process group with ONE bucketed all-reduce. The bucket carries one
    extra element, the number of ranks that failed: a rank whose step raised posts the same
    collective with its flag set and zero gradients (abort_peers), so its peers, blocked in this
    all-reduce, raise PeerFailure instead of waiting for the collective timeout. The
    bucket size is the same on every rank (a parameter without .grad contributes zeros). One host
    read of the flag per update, only when world > 1."""
    if not _distributed(group):
        return
    flat, zeros, flags = _bucket(params)
    parts = [(p.grad if (p.grad is not None and not failed) else zeros[i]).reshape(-1) for i, p in enumerate(params)]
    torch.cat(parts + [flags[1 if failed else 0]], out=flat)
    dist.all_reduce(flat, group=group)
    nfail = int(round(float(flat[-1].item())))
    if nfail:
        raise PeerFailure(f"{nfail} of {dist.get_world_size(group)} data-parallel ranks failed; every rank stops")
    flat = flat[:-1].div_(dist.get_world_size(group))
    off = 0
    for p in params:
        n = p.numel()
        if p.grad is not None:
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
        off += n


def abort_peers(params, group=None):
    """Called by a rank whose training step raised: posts the gradient exchange its peers wait in (or
    will reach next) with the failure flag set. Returns without raising; no-op in a single process."""
    try:
        allreduce_gradients(params, group, failed=True)
    except PeerFailure:
        pass


def finish_sync(params, group=None, failed=False):
    """End of the training loop on every rank: one more exchange of the same shape, so a rank that
    failed after its peers' last update still meets them (PeerFailure on every rank if any failed)."""
    allreduce_gradients(params, group, failed=failed)


DIST_TIMEOUT_S = float(os.environ.get("GM_DIST_TIMEOUT", "900"))


def init_distributed(use_gpu=True):
    """One process per GPU under a launcher (torch.distributed.run sets RANK / WORLD_SIZE /
    LOCAL_RANK; the reference runs independent jobs per GPU, scripts/start_routing_netmon_runs.sh:50).
    Returns (rank, world, local_rank); world 1 initialises nothing. Backend: RCCL ("nccl") with rank
    r on cuda:LOCAL_RANK; gloo when use_gpu is False (CPU tests) or when GM_DIST_SHARE_GPU=1 (every
    rank on cuda:0: a one-GPU rehearsal). A node that shows fewer GPUs than local ranks is an error
    (round 4 fell back to gloo on one GPU silently). Every collective times out after
    GM_DIST_TIMEOUT seconds (default 900). Counting devices does not initialise the GPU."""
    import datetime

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        return 0, 1, 0
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), local
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    share = os.environ.get("GM_DIST_SHARE_GPU") == "1"
    timeout = datetime.timedelta(seconds=DIST_TIMEOUT_S)
    if use_gpu and not share and torch.cuda.device_count() < local_world:
        raise RuntimeError(f"{local_world} local ranks but {torch.cuda.device_count()} visible GPUs: one rank per GPU "
                           "(check HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES), or GM_DIST_SHARE_GPU=1 for a "
                           "one-GPU rehearsal over gloo")
    if not use_gpu:
        dist.init_process_group("gloo", timeout=timeout)
    elif share:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", timeout=timeout)
    else:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    return dist.get_rank(), dist.get_world_size(), local


def shard_seeds(rank, world, n_env, base=0):
    """Per-env numpy-legacy seeds of one rank's env shard: disjoint across ranks."""
    return [(base + rank * n_env + i) & 0xFFFFFFFF for i in range(n_env)]


def broadcast_parameters(modules, src=0, group=None):
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    for m in modules:
        for t in list(m.parameters()) + list(m.buffers()):
            dist.broadcast(t.data, src=src, group=group)


@torch.no_grad()
def interpolate_model(a, b, a_weight, target):
    """src/util.py:8-23: target <- a_weight * a + (1 - a_weight) * b (all state entries)."""
    sa, sb, st = a.state_dict(), b.state_dict(), target.state_dict()
    for k in sa:
        st[k].copy_(a_weight * sa[k] + (1 - a_weight) * sb[k])


# the no-grad target pass on the fused rollout kernels (False: NetMon.forward_graph + joint obs)
FUSED_TARGET = True


def joint_obs(env_obs, network_obs):
    """[env obs | NetMon graph obs] as a view of a buffer whose rows are padded to a multiple of 4
    floats, so the DQN's first GEMM reads it in place (16-byte rows) instead of a padded copy."""
    w = env_obs.shape[-1] + network_obs.shape[-1]
    pad = (w + 3) // 4 * 4 - w
    if pad == 0:
        return torch.cat([env_obs, network_obs], -1)
    z = env_obs.new_zeros(*env_obs.shape[:-1], pad)
    return torch.cat([env_obs, network_obs, z], -1)[..., :w]


def attention_kl(att_weights, tar_att_weights, done):
    """DGN attention regularisation (src/main.py:924-954): KL(softmax(target weights) ||
    softmax(online weights)) per source agent, summed over layers, heads and destination
    agents, averaged over the agents that are not done."""
    attention = F.log_softmax(torch.stack(att_weights), dim=-1)
    target_attention = F.softmax(torch.stack(tar_att_weights), dim=-1)
    shape = attention.shape  # (layers, batch, heads, agents, agents)
    n = shape[-1]
    kl = F.kl_div(attention.reshape(-1, n), target_attention.reshape(-1, n), reduction="none").view(shape)
    kl = kl.transpose(0, -2).transpose(0, 1).sum(dim=(-1, -2, -3))
    return (kl * ~done).sum() / torch.clamp((~done).sum(), min=1)


def _fused_target_ok(netmon, model_tar):
    """The no-grad target pass can run the rollout's fused kernels (fused.netmon_step +
    fused.dqn_q) under the same conditions as a fused NetMonWrapper with a DQN."""
    from . import fused as FU
    from .model import DQN

    return netmon is not None and isinstance(model_tar, DQN) and FU.fused_ok(netmon)


@torch.no_grad()
def _fused_next_q(netmon, model_tar, next_obs, next_node_obs, nbr, next_agent_node, state):
    """Q_target(next obs) [B, A, actions] without materialising the joint next observation:
    the NetMon step on the next node observations (continuing from `state`, the online NetMon
    state after the step) and the target DQN with the readout gathered inside its first GEMM
    (the rollout's path). netmon.state is left as it was."""
    from . import fused as FU

    B, A, od = next_obs.shape
    odp = (od + 3) // 4 * 4  # 16-byte rows for the GEMM's dense source
    env_obs = next_obs.contiguous() if odp == od else F.pad(next_obs, (0, odp - od))
    keep = netmon.save_state()
    st, h_prev = FU.netmon_step(netmon, next_node_obs, nbr.contiguous(), state.detach().contiguous())
    netmon.restore_state(keep)
    dev = env_obs.device
    q = FU.dqn_q(model_tar, env_obs, od, st, h_prev, nbr.contiguous(), next_agent_node.contiguous(),
                 lambda i, m, n: torch.empty(m, n, device=dev), hidden=netmon.hidden_features)
    return q.view(B, A, -1)


class _StateRows:
    """A NetMon state held as its (h, c) rows [B*N, H] (NetMon.state_hc), detached; full() is the
    [B, N, 2H] tensor, [r] the rows of the samples r stacked ([len(r), N, 2H])."""

    def __init__(self, hc):
        h, c, self.B, self.N = hc
        self.h, self.c = h.detach(), c.detach()

    def full(self):
        return torch.stack((self.h, self.c), 1).reshape(self.B, self.N, -1)

    def __getitem__(self, r):
        H = self.h.shape[-1]
        return torch.stack((self.h.view(self.B, self.N, H)[r], self.c.view(self.B, self.N, H)[r]), 2).reshape(
            len(r), self.N, 2 * H)


@torch.no_grad()
def _reused_next_q(netmon, model_tar, batches, joints, states):
    """max_a Q_target(next obs) for every step of a sequence of CONSECUTIVE transitions
    (replay sequences): for t < L-1 the next observation of step t is the observation of step
    t + 1 and the target NetMon (the online NetMon without gradient, continuing from the online
    state after step t) is exactly the online NetMon step t + 1 — unless the episode ended at
    t, where the online state was reset. So the target DQN runs on the online joint observation
    of step t + 1, and only the samples whose episode ended at t (and the last step) get their
    own NetMon step on the stored next observation (src/main.py:878-915 evaluated per step)."""
    L_ = len(batches)
    ep = torch.stack([b.episode_done.expand(b.obs.shape[0]) if b.episode_done.dim() == 0 else b.episode_done
                      for b in batches[:-1]]) if L_ > 1 else None
    done_rows = ep.nonzero().cpu() if ep is not None else None  # one host read per update
    out = []
    for t, batch in enumerate(batches):
        if t == L_ - 1:
            st_t = states[t].full() if isinstance(states[t], _StateRows) else states[t]
            q = _fused_next_q(netmon, model_tar, batch.next_obs, batch.next_node_obs, batch.nbr,
                              batch.next_agent_node, st_t)
            out.append(q.max(dim=2)[0])
            continue
        x = joints[t + 1]
        if isinstance(x, tuple):  # (env obs, graph obs): the two-source first layer
            from . import fused as FU

            env_obs, graph = x
            B, A = env_obs.shape[:2]
            dev = graph.device
            q = FU.dqn_q_dense(model_tar, env_obs, graph, lambda i, m, n: torch.empty(m, n, device=dev))
        else:
            B, A, w = x.shape
            x2 = x.reshape(B * A, w)
            dev = x.device
            q = model_tar.forward_rows(x2, x2.stride(0), w, lambda i, m, n: torch.empty(m, n, device=dev))
        qmax = q.view(B, A, -1).max(dim=2)[0]
        rows = done_rows[done_rows[:, 0] == t, 1]
        if len(rows):
            r = rows.to(dev)
            sub = _fused_next_q(netmon, model_tar, batch.next_obs[r], batch.next_node_obs[r], batch.nbr[r],
                                batch.next_agent_node[r], states[t][r])
            qmax[r] = sub.max(dim=2)[0]
        out.append(qmax)
    return out


def dqn_loss(netmon, model, model_tar, batches, gamma, att_coeff=0.0, aux_model=None, aux_coeff=0.0, parts=None,
             consecutive=False):
    """Sequence loss of src/main.py:840-1000 for DQN / DGN / DQNR / CommNet; netmon may be None.
    Recurrent models start from the stored agent state, the target model runs from the online
    model's next state, and the state is reset for done agents and at episode ends. aux_model
    (with netmon): the NetMon aux head on the new NetMon state, MSE against the stored node aux
    targets, weighted by aux_coeff (src/main.py:586-594, 868-875, 996-1000). consecutive: the
    batches are a replay sequence (step t + 1 continues step t; ReplayBuffer.get_batch), which
    lets the target pass reuse the online NetMon steps (_reused_next_q). parts (a dict) receives
    the loss terms. Returns (loss, list of q, list of q_target)."""
    L = len(batches)
    has_state = hasattr(model, "state")
    loss_q = loss_att = loss_aux = None
    qs, qts = [], []
    last_state = last_ep_done = last_hc = None
    fused_tar = not has_state and _fused_target_ok(netmon, model_tar) and FUSED_TARGET
    reuse = fused_tar and consecutive and att_coeff == 0
    # DQN on NetMon: the first layer reads the env obs and the graph obs as two GEMM sources
    split = netmon is not None and type(model).__name__ == "DQN" and hasattr(model, "forward_split")
    joints, states, next_max = [], [], []
    if not reuse:  # lazily gathered next-step fields (ReplayBuffer.get_batch(lazy_next=True)) in full
        from .replaybuffer import materialize

        batches = [b._replace(next_obs=materialize(b.next_obs), next_node_obs=materialize(b.next_node_obs),
                              next_agent_node=materialize(b.next_agent_node), next_adj=materialize(b.next_adj))
                   for b in batches]
    for t, batch in enumerate(batches):
        if has_state and t == 0:
            model.state = batch.agent_state
        if netmon is None:
            obs, next_obs = batch.obs, batch.next_obs
        else:
            if t == 0:
                netmon.state = batch.node_state
            elif last_hc is not None:  # (h, c) rows: mask them apart, no stacked state
                h_, c_, B_, N_ = last_hc
                m = (~last_ep_done).repeat_interleave(N_).view(-1, 1)
                netmon.set_state_hc(h_ * m, c_ * m, B_, N_)
            else:
                netmon.state = last_state * (~last_ep_done).view(-1, 1, 1)
            graph = netmon.forward_graph(batch.node_obs, batch.nbr, batch.agent_node)
            obs = (batch.obs, graph) if split else joint_obs(batch.obs, graph)
            if aux_model is not None:
                term = torch.mean((aux_model(netmon.state) - batch.node_aux) ** 2) / L
                loss_aux = term if loss_aux is None else loss_aux + term
            last_hc = netmon.state_hc()
            last_state = netmon.state if last_hc is None else None
            last_ep_done = batch.episode_done.expand(batch.obs.shape[0]) if batch.episode_done.dim() == 0 \
                else batch.episode_done
            next_obs = None
        q = model.forward_split(*obs) if split else model(obs, batch.adj)
        qs.append(q)
        if reuse:  # targets after the online pass over the whole sequence
            joints.append((obs[0], obs[1].detach()) if split else obs.detach())
            states.append(_StateRows(last_hc) if last_hc is not None else last_state.detach())
            continue
        with torch.no_grad():
            if has_state:
                model_tar.state = model.state.detach()
            if fused_tar:
                hc = netmon.state_hc()
                st_now = _StateRows(hc).full() if hc is not None else netmon.state
                next_q_max = _fused_next_q(netmon, model_tar, batch.next_obs, batch.next_node_obs, batch.nbr,
                                           batch.next_agent_node, st_now).max(dim=2)[0]
            else:
                if netmon is not None:
                    nno = netmon.forward_graph(batch.next_node_obs, batch.nbr, batch.next_agent_node)
                    next_obs = joint_obs(batch.next_obs, nno)
                next_q_max = model_tar(next_obs, batch.next_adj).max(dim=2)[0]
        next_max.append(next_q_max)
        if has_state:
            ep = batch.episode_done.expand(batch.obs.shape[0]) if batch.episode_done.dim() == 0 \
                else batch.episode_done
            model.state = model.state * (~batch.done * (~ep).view(-1, 1)).unsqueeze(-1)
        if att_coeff > 0 and hasattr(model, "att_weights"):
            kl = attention_kl(model.att_weights, model_tar.att_weights, batch.done) / L
            loss_att = kl if loss_att is None else loss_att + kl
    if reuse:
        next_max = _reused_next_q(netmon, model_tar, batches, joints, states)
    for t, batch in enumerate(batches):
        q = qs[t]
        target = batch.reward + (~batch.done) * gamma * next_max[t]
        q_target = torch.scatter(q.detach(), -1, batch.action.unsqueeze(-1), target.unsqueeze(-1))
        term = torch.mean((q - q_target).pow(2)) / L
        loss_q = term if loss_q is None else loss_q + term
        qts.append(q_target)
    loss = loss_q if loss_att is None else loss_q + att_coeff * loss_att
    if loss_aux is not None:
        loss = loss + aux_coeff * loss_aux
    if parts is not None:
        parts.update(loss_q=loss_q, loss_att=loss_att, loss_aux=loss_aux)
    return loss, qs, qts


def dqn_update(netmon, model, model_tar, optimizer, params, batches, gamma, tau, target_update_steps=0,
               iteration=1, group=None, att_coeff=0.0, aux_model=None, aux_coeff=0.0, parts=None, consecutive=False):
    """One update (src/main.py:840-1026). params must include aux_model's parameters when
    the aux loss is on (src/main.py:594)."""
    loss, qs, qts = dqn_loss(netmon, model, model_tar, batches, gamma, att_coeff, aux_model, aux_coeff, parts,
                             consecutive)
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
    GL.check_range()  # split-f16 range guard of the launches that have finished (no sync)
    return loss.detach(), qs, qts
