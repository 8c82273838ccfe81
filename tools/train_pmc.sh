#!/bin/bash
# HBM bytes of the training kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over a short
# rollout + 2 sequence-batched updates -> gpurun_out/tpmc/summary.txt (per kernel and grid: mean duration
# from the fetch pass, mean read bytes with the gfx950 2x FETCH_SIZE correction, mean written bytes)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/tpmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -T --output-format csv -d gpurun_out/tpmc -o $c \
        -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timers --no-f32-compare --no-pmc \
        --no-extras --graph 0 --train-steps 2 > gpurun_out/tpmc/bench_$c.log 2>&1 || exit $?
done
python - <<'PY' > gpurun_out/tpmc/summary.txt
import csv, collections
def load(c):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/tpmc/{c}_counter_collection.csv")):
        g = r.get("Grid_Size") or r.get("Grid_Size_X")
        dur = int(r.get("End_Timestamp", 0) or 0) - int(r.get("Start_Timestamp", 0) or 0)
        d[(r["Kernel_Name"][:90], int(g))].append((float(r["Counter_Value"]) * 1024, dur))
    return d
f, w = load("FETCH_SIZE"), load("WRITE_SIZE")
rows = []
for k, v in f.items():
    if k[1] < 500000:
        continue
    rd = 2 * sum(x for x, _ in v) / len(v)
    du = sum(y for _, y in v) / len(v)
    wr = sum(x for x, _ in w.get(k, [(0, 0)])) / max(len(w.get(k, [])), 1)
    rows.append((du * len(v), k, len(v), du, rd, wr))
for tot, k, n, du, rd, wr in sorted(rows, reverse=True)[:40]:
    print(f"{k[0][:80]:80s} grid {k[1]:9d} n {n:3d} avg {du / 1e3:9.1f} us  read {rd / 1e6:9.1f} MB  write {wr / 1e6:9.1f} MB  "
          f"{(rd + wr) / max(du, 1):7.1f} GB/s")
PY
