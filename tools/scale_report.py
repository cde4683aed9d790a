#!/usr/bin/env python3
"""What the first node record says, in DESIGN.md §10's order.

  python tools/scale_report.py SCALE_rNN.json [BENCH_or_other.json ...]

Finds every N > 1 bench line in the files (any nesting: a line is a dict
with "metric", "n_gpus" > 1 and "config") and prints, per line:
  1. the node gate's verdicts (hand-off it left, failed paths, disabled
     direct variants) -- a step-down means the faster hand-off was wrong over
     xGMI on that node;
  2. the headline: algbw, roofline against the spec and the calibrated peak;
  3. the transport autotune table and every mode rejected before timing;
  4. the depth-A table (reference_driven) and the one-process service model
     next to the line's value;
  5. the budget: each leg's wall time or skip, and the slowest rank's
     connect (+ gate) time.
Direct thresholds: tools/recommend_direct.py on the same files.
"""
import json
import sys

GATE_BITS = {0x1: "ring uncached", 0x2: "ring release", 0x4: "ring system", 0x8: "LL", 0x10: "one-shot",
             0x20: "two-shot", 0x40: "no peer atomics"}
FIFO = {0: "uncached (relaxed)", 1: "cached + system fences", 2: "uncached + release"}


def bench_lines(obj):
    """Every N > 1 bench line inside a parsed JSON value."""
    if isinstance(obj, dict):
        if "metric" in obj and isinstance(obj.get("n_gpus"), int) and obj["n_gpus"] > 1 and "config" in obj:
            yield obj
            return
        for v in obj.values():
            yield from bench_lines(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from bench_lines(v)


def load(path):
    txt = open(path).read().strip()
    try:
        yield from bench_lines(json.loads(txt))
        return
    except ValueError:
        pass
    for l in txt.splitlines():
        l = l.strip()
        if l.startswith("{"):
            try:
                yield from bench_lines(json.loads(l))
            except ValueError:
                pass


def bits(v):
    return ", ".join(name for b, name in GATE_BITS.items() if v & b) or "none"


def report(line) -> list[str]:
    c = line["config"]
    out = [f"== N = {line['n_gpus']}  {c.get('workload', '')}"]
    g = c.get("node_gate")
    if g:
        out.append(f"1. node gate: ran={g.get('ran')} hand-off={FIFO.get(g.get('fifo_memory_run'), '?')} "
                   f"failed=[{bits(g.get('failed_bits', 0))}] disabled=[{bits(g.get('disabled_bits', 0))}]")
        if g.get("failed_bits", 0) & 0x7:
            out.append("   -> the ring stepped down on this node: make that hand-off the node default (DESIGN §10.1)")
    rf = line.get("roofline", {})
    s = f"2. value {line['value']} {line['unit']} ({line['ms_per_step']} ms); roofline {rf.get('bound')} " \
        f"frac {rf.get('frac')} of {rf.get('peak')} {rf.get('unit')}"
    if "peak_calibrated" in rf:
        s += f"; calibrated peak {rf['peak_calibrated']} -> frac {rf.get('frac_calibrated')}"
    out.append(s)
    tt = c.get("transport_autotune") or []
    timed = [r for r in tt if "ms_per_step" in r]
    if timed:
        best = min(timed, key=lambda r: r["ms_per_step"])
        out.append(f"3. autotune: {len(timed)} timed, best {best['mode']} ch={best.get('channels')} "
                   f"lanes={best.get('lanes')} {best['ms_per_step']} ms; line mode {c.get('fifo_mode')}")
    skipped = [r["mode"] for r in tt if r.get("skipped")]
    if skipped:
        out.append(f"   autotune candidates skipped by the budget: {skipped}")
    for r in c.get("rejected_before_timing") or []:
        out.append(f"   rejected before timing: {r.get('mode')} ({r.get('rank0_reason') or 'failed on another rank'})")
    rd = (c.get("reference_driven") or {}).get("variants") or []
    good = [v for v in rd if v.get("algbw_GBps")]
    if good:
        top = max(good, key=lambda v: v["algbw_GBps"])
        out.append(f"4. depth A: {len(good)}/{len(rd)} variants timed; best {top['variant']} {top['algbw_GBps']} GB/s; "
                   + "; ".join(f"{v['variant']} {v['algbw_GBps']}" for v in good))
    bad = [v for v in rd if v.get("error") or v.get("exact") is False]
    for v in bad:
        out.append(f"   depth A {v.get('variant')}: {v.get('error') or 'not exact'}")
    ip = c.get("in_process_multi_device")
    if ip:
        out.append(f"   one-process service model: {ip.get('algbw_GBps', ip)}")
    b = c.get("budget")
    if b:
        legs = b.get("legs", {})
        sk = [k for k, v in legs.items() if v.get("skipped")]
        slow = sorted(((v["wall_s"], k) for k, v in legs.items() if "wall_s" in v), reverse=True)[:4]
        out.append(f"5. budget {b.get('budget_s')} s, used {b.get('elapsed_s')} s; slowest legs "
                   + ", ".join(f"{k} {w} s" for w, k in slow) + (f"; skipped {sk}" if sk else ""))
    ct = [t for t in c.get("connect_timing_per_rank") or [] if t]
    if ct:
        worst = max(ct, key=lambda t: t.get("connect_s", 0))
        out.append(f"   slowest connect (+ gate): {worst.get('connect_s')} s; handle exchange up to "
                   f"{max(t.get('exchange_s', 0) for t in ct)} s")
    return out


def main():
    n = 0
    for path in sys.argv[1:]:
        for line in load(path):
            n += 1
            print("\n".join(report(line)))
    if n == 0:
        print("no N > 1 bench line found")


if __name__ == "__main__":
    main()
