#!/usr/bin/env python3
"""Direct-kernel thresholds from a node's bench lines.

  python tools/recommend_direct.py SCALE_or_BENCH.json [...]

Reads every N > 1 bench line (one JSON object per line, or a JSON list) and,
from its `config.direct_sweep_fp16` table (ring / two-shot / one-shot per
call at the sweep's sizes, graph replay), prints per N the largest size at
which the LL one-shot is the fastest of all, the largest at which one-shot
is the fastest of ring / two-shot / one-shot and the largest at which
two-shot still beats the ring -- the values to put into default_ll_bytes /
default_oneshot_bytes / default_direct_bytes (mccs_amd/csrc/host/api.cpp)
-- next to the defaults the run used.
"""
import json
import sys


def lines(path):
    txt = open(path).read().strip()
    try:
        whole = json.loads(txt)  # one (indented) object or a list of them
        yield from (whole if isinstance(whole, list) else [whole])
        return
    except ValueError:
        pass
    for l in txt.splitlines():
        l = l.strip()
        if l.startswith("{"):
            try:
                yield json.loads(l)
            except ValueError:
                pass


def recommend(sweep):
    rows = sweep.get("rows", [])
    ll = oneshot = direct = 0
    for r in rows:
        ring = r.get("ring_graph_us", r.get("ring_us"))
        d = r.get("direct_graph_us", r.get("direct_us"))
        o = r.get("oneshot_graph_us", r.get("oneshot_us"))
        q = r.get("ll_graph_us", r.get("ll_us"))
        if ring is None:
            continue
        others = [x for x in (ring, d, o) if x is not None]
        if q is not None and q <= min(others):
            ll = r["bytes"]
        if o is not None and o <= min(ring, d if d is not None else ring):
            oneshot = r["bytes"]
        if d is not None and d < ring:
            direct = r["bytes"]
    return ll, oneshot, direct


def main(paths):
    for p in paths:
        for d in lines(p):
            sweep = (d.get("config") or {}).get("direct_sweep_fp16")
            if not sweep:
                continue
            q, o, t = recommend(sweep)
            used = (sweep.get("summary") or {}).get("default_thresholds")
            print(json.dumps({"file": p, "n_gpus": d.get("n_gpus"), "p2p_atomics": sweep.get("p2p_atomics"),
                              "failed": sweep.get("failed"), "recommend_ll_bytes": q, "recommend_oneshot_bytes": o,
                              "recommend_direct_bytes": t, "defaults_used": used}))


if __name__ == "__main__":
    main(sys.argv[1:])
