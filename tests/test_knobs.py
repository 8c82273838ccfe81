"""The environment variables the product reads (non-default kernel paths behind run-time
knobs that no long-horizon test ran were removed). The package and its HIP sources may read only these;
bench.py adds its own launch / rehearsal switches. A new knob must be added here on purpose, with a test
that runs the path it selects."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"""(?:os\.environ\.get\(|os\.environ\[|getenv\()\s*["']([A-Z0-9_]+)["']""")

PACKAGE_KNOBS = {
    "GM_GEMM",            # x3 (split-f16, default) | f32: both GEMM forms run every long-horizon case
    "GM_LIB",             # load another build of the library (A/B of two builds in one process)
    "GM_DIST_TIMEOUT",    # collective timeout of the data-parallel process group
    "GM_DIST_SHARE_GPU",  # one-GPU rehearsal of the N-rank path (gloo)
    "GM_FAULT",           # main.py failure injection (tests/test_distributed*.py)
}
BENCH_KNOBS = {"GM_BENCH_RAISE", "GM_BENCH_SHARE_GPU", "GM_DIST_TIMEOUT"}


def _reads(paths):
    found = {}
    for p in paths:
        with open(p, errors="replace") as f:
            for name in PAT.findall(f.read()):
                found.setdefault(name, set()).add(os.path.relpath(p, ROOT))
    return found


def test_package_reads_only_the_listed_knobs():
    pkg = os.path.join(ROOT, "graph-marl_amd")
    files = glob.glob(os.path.join(pkg, "*.py")) + glob.glob(os.path.join(pkg, "csrc", "*"))
    found = _reads(files)
    gm = {k: v for k, v in found.items() if k.startswith("GM_")}
    assert set(gm) == PACKAGE_KNOBS, gm


def test_bench_reads_only_the_listed_knobs():
    found = _reads([os.path.join(ROOT, "bench.py")])
    assert {k for k in found if k.startswith("GM_")} == BENCH_KNOBS, found
