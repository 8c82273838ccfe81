"""CPU tests of the C-ABI boundary: the shared library loads and exports every
entry point include/graph_marl_amd.h declares (no compute without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "graph_marl_amd.h")
TUNING = os.path.join(ROOT, "include", "graph_marl_amd_tuning.h")


def declared_functions(path=None):
    if path is None:
        return declared_functions(HEADER) | declared_functions(TUNING)
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(gm_[a-z0-9_]+)\s*\(", txt))


def test_header_and_binding_agree(gm):
    assert declared_functions(HEADER) == set(gm._lib.EXPORTS)
    assert declared_functions(TUNING) == set(gm._lib.TUNING_EXPORTS)


def test_library_was_built_from_these_sources(gm):
    """gm_build_info() carries the SHA-256 of the sources the library was linked from: a stale
    in-tree .so (sources edited, library not rebuilt) fails here."""
    info = gm._lib.build_info()
    assert info["arch"] == "gfx950"
    assert info["src"] == gm._lib.source_hash(), f"library built from other sources: {info}"


def test_library_reports_only_the_supported_forms(gm):
    """Round 5 pruned the GEMM variant knobs: the library reports the one split
    form it carries (x3=lo12: the A operand's low piece scaled by 2^12 in every kernel, pinned at the
    production tiles by tests/test_gemm_precision_gpu.py) and the product build (diag=0); the only
    compile-time switch left in gm_gemm.hip is the GM_DIAG stamp build, and the removed forms (the
    bare asm split that raced the MFMA read, the unscaled low piece, the neutral tile / priority /
    stage variants) are gone from the source."""
    info = gm._lib.build_info()
    assert info.get("x3") == "lo12" and info.get("diag") == "0", info
    assert set(info) == {"src", "arch", "hipcc", "x3", "diag", "matches_tree"}, info
    src = open(os.path.join(ROOT, "graph-marl_amd", "csrc", "gm_gemm.hip")).read()
    assert set(re.findall(r"#ifndef (GM_\w+)", src)) == {"GM_DIAG"}
    for gone in ("GM_SPLIT_ASM", "GM_ROLLOUT_LO_UNSCALED", "GM_FWD_LO_UNSCALED", "GM_NARROW_TILE", "GM_PRIO",
                 "GM_READOUT_TILE", "GM_HEAD_STAGES", "GM_PINGPONG", "asm(\"v_fma_mix"):
        assert gone not in src, gone
    for f in ("gm_netmon.hip", "gm_env.hip"):
        txt = open(os.path.join(ROOT, "graph-marl_amd", "csrc", f)).read()
        for gone in ("GM_RENC_CPL", "GM_RENC_TPB", "GM_RENC_ROWS"):
            assert gone not in txt, (f, gone)


def test_library_exports_every_declared_symbol(gm):
    path = gm._lib.LIB_PATH
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "graph-marl_amd", "csrc")])
    L = gm._lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", path]).decode()
    syms = set(re.findall(r"\bT (gm_[a-z0-9_]+)\b", out))
    assert declared_functions() <= syms


def test_error_path_without_device(gm):
    """Invalid arguments are rejected before any device call, with a message."""
    L = gm._lib.lib()
    cfg = gm._lib.EnvConfig()
    cfg.n_env, cfg.n_nodes, cfg.n_data, cfg.env_var = 1, 21, 20, 1  # odd node count
    h = ctypes.c_void_p()
    seeds = (ctypes.c_uint32 * 1)(0)
    rc = L.gm_env_create(ctypes.byref(cfg), ctypes.cast(seeds, ctypes.c_void_p), ctypes.byref(h))
    assert rc == -1
    assert b"even" in L.gm_last_error()
    rc = L.gm_linear_f32(None, 0, None, 0, None, 0, 0, 0, 0, None, 0, None)
    assert rc == -1


def test_product_refuses_cpu(gm):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(gm._lib.GMError):
        gm.Routing(gm.Network(20), n_env=2)


def test_training_entry_points_reject_bad_arguments(gm):
    """The round-2 training entry points validate their arguments before any device call."""
    L = gm._lib.lib()
    vp = ctypes.c_void_p
    assert L.gm_gemm_set_dgrad(3) == -1 and b"form" in L.gm_last_error()
    assert L.gm_gemm_set_dgrad(-1) == 0
    assert L.gm_gemm_set_wgrad(4) == -1
    assert L.gm_gemm_set_wgrad(-1) == 0
    # gather of 12-byte records (not a multiple of 16) and a null source
    assert L.gm_gather_records(vp(16), 16, 16, vp(16), vp(16), 1, 1, 12, vp(16), None) == -1
    assert b"16-byte" in L.gm_last_error()
    assert L.gm_gather_records(None, 16, 16, vp(16), vp(16), 1, 1, 16, vp(16), None) == -1
    # LSTM cell backward without its operands
    args = gm._lib.LSTMBwdArgs()
    assert L.gm_lstm_cell_bwd(ctypes.byref(args), None) == -1
    # Q-head backward with more than 4 heads
    assert L.gm_qhead_bwd(vp(16), 5, 5, vp(16), 8, vp(16), 8, 8, 8, 1, vp(16), 8, vp(16), vp(16), vp(16), 8, None,
                          None) == -1


def test_routing_encoder_source_rejects_bad_arguments(gm):
    """gm_encoder_x3 and the ROUTING_ENC A source (round 5) validate before any device call: the source
    mode, the layer widths (256 -> 128), degree 3, 4N + 8 <= 208 and whole 32-wide k tiles; gm_gemm_f32
    refuses the source outright."""
    import importlib

    FU = importlib.import_module("graph-marl_amd.fused")
    L = gm._lib.lib()
    FU._setup()
    vp = ctypes.c_void_p

    def src(**kw):
        s = FU.ASrc()
        s.mode, s.p0, s.p1, s.ld0, s.ld1, s.nbr = FU.GM_A_ROUTING_ENC, 16, 16, 88, 512, 16
        s.n_nodes, s.deg, s.k, s.bias0, s.act0 = 20, 3, 512, 16, 1
        for k, v in kw.items():
            setattr(s, k, v)
        return s

    def chain(s, n2=256, n3=128, m=81920):
        return L.gm_encoder_x3(ctypes.byref(s), vp(16), vp(16), vp(16), 1, vp(16), vp(16), vp(16), 1, m, n2, n3,
                               vp(16), 128, None)

    assert chain(src(), n2=512) == -1 and b"256, 128" in L.gm_last_error()
    assert chain(src(), n3=64) == -1
    assert chain(src(mode=FU.GM_A_DENSE)) == -1 and b"routing-encoder" in L.gm_last_error()
    for bad in (dict(deg=4), dict(n_nodes=51), dict(k=500), dict(nbr=None)):
        assert chain(src(**bad)) != 0, bad
        assert b"routing-encoder" in L.gm_last_error(), bad
    assert chain(src(), m=81919) != 0  # rows not whole graphs
    s = src()
    assert L.gm_gemm_f32(ctypes.byref(s), None, vp(16), 512, vp(16), 81920, 256, 1, vp(16), 256, None, 0, None, 0,
                         None, None) != 0
