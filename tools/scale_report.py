#!/usr/bin/env python3
"""Tabulate the N > 1 bench lines of a scaling run (the driver's SCALE_rNN.json,
or any files holding bench.py JSON lines) as markdown: per N the headline
(strong: configs[3]'s 1 GiB job over N GPUs) and the weak 256 MiB-per-GPU
reading with their per-GPU roofline fractions, then each switch path's time
per all-reduce, its fraction of the xGMI bound and its phases — the numbers
DESIGN.md §10 says to act on once a real node has run.  Reads any JSON: every
object carrying "n_gpus" and "metric" counts as a bench line (also lines
embedded in text logs).  Usage: scale_report.py FILE [FILE ...]"""
import json
import re
import sys

SWITCHES = ("switchsim", "p2p_switch", "xgmi_switch", "xgmi_switch_push", "rccl_fp32_allreduce")


def bench_lines(obj):
    """Every bench line (dict with n_gpus + metric) inside obj, depth-first."""
    if isinstance(obj, dict):
        if "n_gpus" in obj and "metric" in obj:
            yield obj
            return
        for v in obj.values():
            yield from bench_lines(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from bench_lines(v)


def load(path):
    text = open(path).read()
    try:
        yield from bench_lines(json.loads(text))
        return
    except json.JSONDecodeError:
        pass
    for line in text.splitlines():                     # a log with JSON lines in it
        m = re.search(r"\{.*\}\s*$", line)
        if m:
            try:
                yield from bench_lines(json.loads(m.group(0)))
            except json.JSONDecodeError:
                continue


def fmt(v, nd=3):
    if v is None:
        return "–"
    return f"{v:.{nd}f}" if isinstance(v, float) else str(v)


def report(lines):
    lines = sorted(lines, key=lambda b: b["n_gpus"])
    out = ["| N | value (GB/s) | frac / GPU | ms/step | weak 256 MiB (GB/s) | weak frac / GPU | self_check |",
           "|---|---|---|---|---|---|---|"]
    for b in lines:
        wk = b.get("weak_256MiB") or {}
        out.append(f"| {b['n_gpus']} | {fmt(b.get('value'), 1)} | {fmt((b.get('roofline') or {}).get('frac'))} | "
                   f"{fmt(b.get('ms_per_step'), 5)} | {fmt(b.get('weak_256MiB_value'), 1)} | "
                   f"{fmt((wk.get('roofline') or {}).get('frac'))} | {b.get('self_check')} |")
    base = next((b for b in lines if b["n_gpus"] == 1), None)
    if base:
        out += ["", "Scaling of `value` against N = 1 (strong; the driver computes its own):", ""]
        out += ["| N | value / (N x value(1)) |", "|---|---|"]
        for b in lines:
            out.append(f"| {b['n_gpus']} | {fmt(b['value'] / (b['n_gpus'] * base['value']))} |")
    out += ["", "| N | path | ms / all-reduce | busbw GB/s | frac of xGMI bound | verified | phases (ms) |",
            "|---|---|---|---|---|---|---|"]
    for b in lines:
        for k in SWITCHES:
            f = b.get(k) or (b.get("side") or {}).get(k)
            if not f:
                continue
            ph = ", ".join(f"{p} {fmt(t, 2)}" for p, t in (f.get("phases_ms") or {}).items())
            out.append(f"| {b['n_gpus']} | {k} | {fmt(f.get('ms_per_allreduce'))} | {fmt(f.get('busbw_GBps'), 2)} | "
                       f"{fmt(f.get('frac_of_xgmi_bound'), 4)} | {f.get('verified', '–')} | {ph or f.get('error', '–')} |")
    fails = [(b["n_gpus"], b.get("failures"), b.get("diagnostic_failures")) for b in lines
             if b.get("failures") or b.get("diagnostic_failures")]
    if fails:
        out += ["", "Failures:", ""] + [f"* N = {n}: fatal {f}, diagnostic {d}" for n, f, d in fails]
    return "\n".join(out)


def main(paths):
    lines = [b for p in paths for b in load(p)]
    if not lines:
        sys.exit("no bench lines found")
    print(report(lines))


if __name__ == "__main__":
    main(sys.argv[1:])
