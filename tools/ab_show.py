#!/usr/bin/env python3
"""Prints value / roofline / selected kernel times of bench.py logs: python tools/ab_show.py LOG..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    ks = d.get("kernels", {})
    sel = {k.split(":")[0] + ":" + k.split(":")[-1]: round(v["avg_us"], 1) for k, v in ks.items() if "avg_us" in v}
    rt = (d.get("rollout_train") or {}).get("value")
    print(f, d["value"], (d.get("roofline") or {}).get("frac"), rt, sel)
