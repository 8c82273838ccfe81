"""ctypes binding of libgraphmarl_amd.so (the C ABI in include/graph_marl_amd.h).

torch is imported first so that the library binds to the HIP runtime torch already
loaded (same libamdhip64.so.7 soname) and torch streams/tensors are usable as
plain hipStream_t / device pointers. There is no CPU fallback: if the library is
missing or no GPU is present the product path raises.
"""
import ctypes as C
import os

import torch  # noqa: F401  (must precede the HIP library load)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GM_LIB") or os.path.join(HERE, "lib", "libgraphmarl_amd.so")

GM_OK = 0
GM_INFO_FIELDS = 9
INFO_KEYS = ["looped", "throughput", "dropped", "blocked", "n_delays", "sum_delays", "n_arrived",
             "sum_delays_arrived", "sum_spr"]
TOPO_FIXED, TOPO_RANDOM, TOPO_LIST, TOPO_SEQUENTIAL = 0, 1, 2, 3
GM_EVAL_FIELDS = 5
EVAL_KEYS = ["total_edge_load", "occupied_edges", "packets_on_edges", "total_packet_size", "sum_packet_distances"]

# every symbol the header declares (checked by tests/test_capi.py)
EXPORTS = [
    "gm_last_error", "gm_version", "gm_env_create", "gm_env_destroy", "gm_env_dims", "gm_env_reset",
    "gm_env_step", "gm_env_observe", "gm_env_topology", "gm_env_final_info", "gm_policy_egreedy", "gm_env_policy_step",
    "gm_env_get_state", "gm_env_set_state", "gm_build_seed_list", "gm_mp_aggregate", "gm_mp_aggregate_rows", "gm_mp_aggregate_bwd", "gm_leaky_bwd", "gm_netmon_readout",
    "gm_netmon_readout_bwd", "gm_lstm_pointwise", "gm_lstm_pointwise_bwd", "gm_linear_f32", "gm_gemm_f32",
    "gm_simple_create", "gm_simple_destroy", "gm_simple_reset", "gm_simple_step",
    "gm_simple_observe", "gm_simple_policy_egreedy", "gm_simple_get_state", "gm_env_set_topology",
    "gm_policy_shortest_path", "gm_env_first_hops", "gm_routing_node_encoder", "gm_gemm_x3", "gm_gemm_x3_head", "gm_absmax_scale", "gm_absmax_scale_rows", "gm_gemm_x3_wgrad", "gm_gemm_x3_wgrad2", "gm_absmax_finish",
    "gm_gemm_pack_x3", "gm_gemm_pack_x3_bytes", "gm_gemm_range_status",
    "gm_pcg64_seed", "gm_pcg64_choice", "gm_lnlstm_pointwise", "gm_agent_attention", "gm_agent_comm",
    "gm_gemm_x3_dgrad", "gm_lstm_cell_bwd", "gm_qhead_bwd", "gm_netmon_readout_ld", "gm_routing_node_encoder_bits", "gm_gather_records",
    "gm_lnlstm_fwd", "gm_lnlstm_bwd", "gm_gru_pointwise", "gm_gru_bwd", "gm_act_bwd", "gm_build_info",
    "gm_act_fwd", "gm_act_bwd_z", "gm_obs_from_gemm", "gm_encoder_x3", "gm_step_mse_blocks", "gm_step_mse",
    "gm_step_mse_bwd",
]
# kernel-form switches (include/graph_marl_amd_tuning.h)
TUNING_EXPORTS = ["gm_gemm_set_tile", "gm_gemm_set_wgrad", "gm_gemm_set_mfma", "gm_gemm_set_dgrad", "gm_gemm_form"]

# Arithmetic form of the fused rollout GEMMs (graph-marl_amd/fused.py): "x3" = split-f16
# MFMA with fp32 accumulation (default), "f32" = exact fp32 MFMA. GM_GEMM=f32 selects the
# exact form process-wide.
GEMM_MODE = os.environ.get("GM_GEMM", "x3")
if GEMM_MODE not in ("x3", "f32"):
    raise ValueError(f"GM_GEMM must be 'x3' or 'f32', not {GEMM_MODE!r}")

class EnvConfig(C.Structure):
    _fields_ = [
        ("n_env", C.c_int32), ("n_nodes", C.c_int32), ("n_data", C.c_int32), ("env_var", C.c_int32),
        ("congestion", C.c_int32), ("action_mask", C.c_int32), ("ttl", C.c_int32), ("topo_mode", C.c_int32),
        ("topo_seed", C.c_int64), ("seed_list", C.POINTER(C.c_int64)), ("n_seed_list", C.c_int32),
        ("excluded", C.POINTER(C.c_int64)), ("n_excluded", C.c_int32), ("device", C.c_int32),
        ("k", C.c_int32),
    ]


class ObsBuffers(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("obs_row_stride", C.c_int64), ("node_obs", C.c_void_p),
                ("agent_node", C.c_void_p), ("agent_adj", C.c_void_p), ("obs_gemm", C.c_void_p),
                ("obs_gemm_stride", C.c_int64)]


class StepDetail(C.Structure):
    _fields_ = [("done_steps", C.c_void_p), ("done_opt", C.c_void_p), ("success", C.c_void_p), ("eval", C.c_void_p)]


class EnvState(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in [
        "now", "target", "edge", "time", "ttl", "start", "spw", "agent_steps", "size", "visited", "amask",
        "loads", "topo_seed", "topo_reps", "edge_a", "edge_b", "edge_len", "nbr_edge", "apsp", "rng_key",
        "rng_pos", "seq_index"]]


class PCG64(C.Structure):
    """gm_pcg64: numpy Generator(PCG64) state (bit_generator.state)."""
    _fields_ = [("state_hi", C.c_uint64), ("state_lo", C.c_uint64), ("inc_hi", C.c_uint64), ("inc_lo", C.c_uint64),
                ("has_uint32", C.c_uint32), ("uinteger", C.c_uint32)]


class LSTMBwdArgs(C.Structure):
    """gm_lstm_bwd_args (include/graph_marl_amd.h)."""
    _fields_ = [
        ("act", C.c_void_p), ("ld_act", C.c_int64), ("c_in", C.c_void_p), ("ld_cin", C.c_int64),
        ("c_out", C.c_void_p), ("ld_cout", C.c_int64), ("dh0", C.c_void_p), ("ld_dh0", C.c_int64),
        ("dh1", C.c_void_p), ("ld_dh1", C.c_int64), ("dm", C.c_void_p), ("ld_dm", C.c_int64),
        ("nbr", C.c_void_p), ("n_nodes", C.c_int32), ("deg", C.c_int32), ("mean", C.c_int32),
        ("dh_ext", C.c_void_p), ("ld_ext", C.c_int64), ("dc_ext", C.c_void_p), ("ld_dcext", C.c_int64),
        ("ext_mask", C.c_void_p), ("rows_per_sample", C.c_int32), ("dc", C.c_void_p), ("ld_dc", C.c_int64),
        ("m", C.c_int32), ("hidden", C.c_int32), ("dgates", C.c_void_p), ("ld_dg", C.c_int64),
        ("dc_out", C.c_void_p), ("ld_dco", C.c_int64), ("bias_part", C.c_void_p), ("rows_per_block", C.c_int32),
        ("dg_scale", C.c_void_p), ("dg_max", C.c_void_p),
    ]


class WgradSrc(C.Structure):
    """gm_wgrad_src (include/graph_marl_amd.h): one B source of gm_gemm_x3_wgrad2 with its row map."""
    _fields_ = [("p", C.c_void_p), ("ld", C.c_int64), ("scale", C.c_void_p), ("period", C.c_int64),
                ("shift", C.c_int64), ("rows", C.c_int64)]


class GMError(RuntimeError):
    pass


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GMError(f"{LIB_PATH} not built: run `make -C graph-marl_amd/csrc` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.gm_last_error.restype = C.c_char_p
    L.gm_env_create.argtypes = [C.POINTER(EnvConfig), vp, C.POINTER(vp)]
    L.gm_env_destroy.argtypes = [vp]
    L.gm_env_dims.argtypes = [vp] + [C.POINTER(i32)] * 5
    L.gm_env_reset.argtypes = [vp, vp, C.POINTER(ObsBuffers), vp]
    L.gm_env_step.argtypes = [vp, vp, vp, vp, vp, C.POINTER(StepDetail), C.POINTER(ObsBuffers), vp]
    L.gm_env_observe.argtypes = [vp, C.POINTER(ObsBuffers), vp]
    L.gm_env_topology.argtypes = [vp, vp, vp, vp, vp, vp]
    L.gm_env_final_info.argtypes = [vp, vp, vp]
    L.gm_policy_egreedy.argtypes = [vp, vp, C.c_double, vp, vp]
    L.gm_env_policy_step.argtypes = [vp, vp, C.c_double, vp, vp, vp, vp, C.POINTER(StepDetail), C.POINTER(ObsBuffers),
                                     vp]
    L.gm_env_get_state.argtypes = [vp, C.POINTER(EnvState)]
    L.gm_env_set_state.argtypes = [vp, C.POINTER(EnvState)]
    L.gm_build_seed_list.argtypes = [i32, i64, i32, vp, i32, i32, vp]
    L.gm_mp_aggregate.argtypes = [vp, vp, i32, i32, i32, i32, i32, vp, vp]
    L.gm_mp_aggregate_rows.argtypes = [vp, C.c_int64, vp, i32, i32, i32, i32, i32, vp, C.c_int64, vp]
    L.gm_leaky_bwd.argtypes = [vp, vp, C.c_int64, i32, C.c_float, vp, vp, i32, vp, vp]
    L.gm_mp_aggregate_bwd.argtypes = [vp, vp, i32, i32, i32, i32, i32, vp, vp]
    L.gm_netmon_readout.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, i64, vp]
    L.gm_netmon_readout_bwd.argtypes = [vp, i64, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp]
    L.gm_lstm_pointwise.argtypes = [vp, vp, i32, i32, vp, vp, vp, vp]
    L.gm_lstm_pointwise_bwd.argtypes = [vp, vp, vp, vp, vp, i32, i32, vp, vp, vp, vp]
    L.gm_linear_f32.argtypes = [vp, i64, vp, i64, vp, i32, i32, i32, i32, vp, i64, vp]
    L.gm_gemm_set_tile.argtypes = [i32]
    L.gm_gemm_set_wgrad.argtypes = [i32]
    L.gm_gemm_set_mfma.argtypes = [i32]
    L.gm_gemm_set_dgrad.argtypes = [i32]
    L.gm_lstm_cell_bwd.argtypes = [C.POINTER(LSTMBwdArgs), vp]
    L.gm_qhead_bwd.argtypes = [vp, i64, i32, vp, i64, vp, i64, i64, i32, i32, vp, i64, vp, vp, vp, i32, vp, vp]
    L.gm_netmon_readout_ld.argtypes = [vp, i64, vp, i64, vp, vp, i32, i32, i32, i32, i32, vp, i64, vp]
    L.gm_routing_node_encoder_bits.argtypes = [vp, i64, vp, i32, i32, vp, vp, i32, i32, vp, i64, vp, i64, vp]
    L.gm_env_set_topology.argtypes = [vp, i32, i64, vp, i32, i32]
    L.gm_policy_shortest_path.argtypes = [vp, vp, vp]
    L.gm_env_first_hops.argtypes = [vp, vp, vp]
    L.gm_agent_attention.argtypes = [vp, vp, vp, i64, vp, i32, i32, i32, i32, i32, vp, i64, vp, vp]
    L.gm_agent_comm.argtypes = [vp, i64, vp, i32, i32, i32, vp, i64, vp]
    L.gm_gemm_pack_x3_bytes.argtypes = [i32, i32]
    L.gm_gemm_pack_x3_bytes.restype = i64
    L.gm_gemm_pack_x3.argtypes = [vp, i64, i32, i32, vp, vp, vp]
    L.gm_routing_node_encoder.argtypes = [vp, i64, vp, i32, i32, vp, vp, i32, i32, vp, i64, vp]
    L.gm_gemm_range_status.argtypes = [C.POINTER(i32), i32]
    L.gm_pcg64_seed.argtypes = [C.c_uint64, C.POINTER(PCG64)]
    L.gm_pcg64_choice.argtypes = [vp, i64, i64, vp, vp]
    L.gm_gather_records.argtypes = [vp, i64, i64, vp, vp, i32, i64, i64, vp, vp]
    L.gm_lnlstm_pointwise.argtypes = [vp, i64, vp, i64] + [vp] * 7 + [i32, i32, C.c_float, vp, i64, vp, i64, vp]
    # round-3 entry points; GM_LIB may name an older build for A-B timing, which lacks them
    newer = {
        "gm_lnlstm_fwd": [vp, i64, vp, i64, vp, i64] + [vp] * 7 + [i32, i32, C.c_float, vp, i64, vp, i64, vp, vp],
        "gm_lnlstm_bwd": [vp, i64, vp, i64, vp, i64] + [vp] * 8 + [vp, i64, vp, i64, i32, i32, i32, vp, i64, vp, i64, vp,
                                                                   i64, vp, vp],
        "gm_gru_pointwise": [vp, i64, vp, i64, vp, i64, i32, i32, vp, i64, vp],
        "gm_gru_bwd": [vp, i64, vp, i64, vp, i64, vp, i64, i32, i32, vp, i64, vp, i64, vp, i64, vp],
        "gm_act_bwd": [vp, vp, C.c_int64, i32, i32, vp, vp, i32, vp, vp],
        "gm_act_fwd": [vp, C.c_int64, i32, i32, vp, vp],
        "gm_act_bwd_z": [vp, vp, C.c_int64, i32, i32, vp, vp, i32, vp, vp],
        "gm_obs_from_gemm": [vp, i64, i64, i32, vp, i64, vp],
        "gm_step_mse_blocks": [i64],
        "gm_step_mse": [vp, vp, i64, i32, vp, vp],
        "gm_step_mse_bwd": [vp, vp, i64, i32, vp, C.c_float, vp, vp],
    }
    for name, at in newer.items():
        if hasattr(L, name) or not os.environ.get("GM_LIB"):
            getattr(L, name).argtypes = at
    if hasattr(L, "gm_step_mse_blocks"):
        L.gm_step_mse_blocks.restype = i32
    if hasattr(L, "gm_build_info"):
        L.gm_build_info.restype = C.c_char_p
    if hasattr(L, "gm_gemm_form"):
        L.gm_gemm_form.restype = C.c_char_p
    _lib = L
    return L


def source_hash():
    """16 hex digits of the SHA-256 of the kernel sources and public headers, in the order the
    Makefile hashes them (byte-sorted csrc/gm_*.hip + gm_*.hpp, then include/*.h)."""
    import glob
    import hashlib

    csrc, inc = os.path.join(HERE, "csrc"), os.path.join(os.path.dirname(HERE), "include")
    files = sorted(glob.glob(os.path.join(csrc, "gm_*.hip")) + glob.glob(os.path.join(csrc, "gm_*.hpp")),
                   key=lambda f: os.path.basename(f).encode())
    files += sorted(glob.glob(os.path.join(inc, "*.h")), key=lambda f: os.path.basename(f).encode())
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info():
    """gm_build_info() of the loaded library as a dict (src, arch, hipcc), plus whether its source
    hash matches the tree's sources (None when the sources are not present)."""
    L = lib()
    if not hasattr(L, "gm_build_info"):
        return {"src": None, "matches_tree": None}
    d = dict(kv.split("=", 1) for kv in L.gm_build_info().decode().split())
    if hasattr(L, "gm_gemm_form"):  # the arithmetic form the GEMM kernels were compiled with
        d.update(kv.split("=", 1) for kv in L.gm_gemm_form().decode().split())
    try:
        d["matches_tree"] = d.get("src") == source_hash()
    except OSError:
        d["matches_tree"] = None
    return d


def check(rc):
    if rc != GM_OK:
        raise GMError(f"graph_marl_amd error {rc}: {lib().gm_last_error().decode()}")


def range_status(clear=False):
    """1 when a finished split-f16 GEMM saw an operand outside the f16 range since the last
    clear (gm_gemm_range_status: a host-mapped word, no stream synchronisation)."""
    v = C.c_int32(0)
    check(lib().gm_gemm_range_status(C.byref(v), int(clear)))
    return v.value


def check_range():
    """Raise GMError when a finished split-f16 GEMM went out of the f16 range: its outputs
    (and everything computed from them) are invalid. Called at the rollout's episode ends
    and after every update; the next gm_gemm_x3 call fails the same way."""
    if GEMM_MODE == "x3" and range_status():
        raise GMError("split-f16 GEMM operand outside the f16 range (|a| >= 2^15 possible): results since the "
                      "last check are invalid; rerun with GM_GEMM=f32")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _tensors(v):
    """Device tensors held by a cached value (tensor, tuple / list, or an object with __slots__)."""
    if isinstance(v, torch.Tensor):
        yield v
    elif isinstance(v, (tuple, list)):
        for x in v:
            yield from _tensors(x)
    elif v is not None and hasattr(v, "__slots__"):
        for s in v.__slots__:
            yield from _tensors(getattr(v, s, None))


class Published:
    """Stream hand-off of a cached device value (packed weights built lazily by whichever stream
    first needs them). The builder's stream records an event right after the value's kernels;
    the first use from any other stream makes that stream wait for the event and registers the
    value's tensors with it (record_stream: their memory is not reused while that stream may still
    read them after the cache drops the value). StreamedRollout's groups share the caches: without
    this, group 1's first GEMM could read a pack group 0's stream had not finished writing."""
    __slots__ = ("ev", "seen")

    def __init__(self):
        s = torch.cuda.current_stream()
        self.seen = {s}
        self.ev = None
        if not torch.cuda.is_current_stream_capturing():
            self.ev = torch.cuda.Event()
            self.ev.record(s)

    def acquire(self, val):
        s = torch.cuda.current_stream()
        if s in self.seen or self.ev is None or torch.cuda.is_current_stream_capturing():
            return  # (a capture starts from a synchronised device: every pack is complete)
        s.wait_event(self.ev)
        for t in _tensors(val):
            t.record_stream(s)
        self.seen.add(s)


def require_gpu():
    if not torch.cuda.is_available():
        raise GMError("graph-marl_amd needs a ROCm GPU (torch.cuda.is_available() is False); there is no CPU path")


# ---------------------------------------------------------------------------
# Optional per-kernel timing (bench.py): when PROF is a dict, every wrapped launch
# records a pair of HIP events on the launch stream under its tag.
# ---------------------------------------------------------------------------
PROF = None
# launch-order recorder (bench.py's PMC child): when TRACE is a list, every wrapped launch appends its tag
TRACE = None


class timed:
    __slots__ = ("tag", "s")

    def __init__(self, tag):
        self.tag = tag
        self.s = None

    def __enter__(self):
        if TRACE is not None and self.tag:
            TRACE.append(self.tag)
        if PROF is not None and self.tag:
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *exc):
        if self.s is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            PROF.setdefault(self.tag, []).append((self.s, e))
        return False
