#!/usr/bin/env python3
"""Tabulate the N > 1 bench lines of a scaling run (the driver's SCALE_rNN.json,
or any files holding bench.py JSON lines) as markdown: per N the two readings
every line carries (value = weak_256MiB_value: 256 MiB buckets on every GPU;
strong_1GiB_value: configs[3]'s 1 GiB job over the N GPUs) with their per-GPU
roofline fractions, the scaling efficiency of EACH reading against the same
reading at N = 1, then each switch path's time
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


READINGS = (("value", "value (= weak_256MiB_value)"), ("weak_256MiB_value", "weak 256 MiB per GPU"),
            ("strong_1GiB_value", "strong 1 GiB job"))


def reading_frac(b, key):
    """The per-GPU roofline fraction of one reading of a line."""
    sub = {"value": b, "weak_256MiB_value": b.get("weak_256MiB") or {},
           "strong_1GiB_value": b.get("strong_1GiB") or {}}[key]
    return (sub.get("roofline") or {}).get("frac")


def efficiency(lines):
    """{reading: {N: rate(N) / (N x rate(1))}} — each reading against the SAME
    reading at N = 1 (never one workload's rate over another's).
    A reading missing at N = 1 or at N gets no entry for that N.  Weak and
    strong readings both ideally scale as N x rate(1) (strong: the job's time
    shrinks N-fold)."""
    base = next((b for b in lines if b["n_gpus"] == 1), None)
    out = {}
    for key, _ in READINGS:
        r1 = base.get(key) if base else None
        out[key] = {b["n_gpus"]: b[key] / (b["n_gpus"] * r1) for b in lines
                    if r1 and isinstance(b.get(key), (int, float))}
    return out


def report(lines):
    lines = sorted(lines, key=lambda b: b["n_gpus"])
    out = ["| N | weak 256 MiB = value (GB/s) | weak frac / GPU | ms/step | strong 1 GiB (GB/s) | "
           "strong frac / GPU | scaling | self_check |",
           "|---|---|---|---|---|---|---|---|"]
    for b in lines:
        st = b.get("strong_1GiB") or {}
        out.append(f"| {b['n_gpus']} | {fmt(b.get('value'), 1)} | {fmt(reading_frac(b, 'value'))} | "
                   f"{fmt(b.get('ms_per_step'), 5)} | {fmt(b.get('strong_1GiB_value'), 1)} | "
                   f"{fmt(reading_frac(b, 'strong_1GiB_value'))} | {b.get('scaling')} | "
                   f"{b.get('self_check')}{'' if st.get('self_check', True) else ' (strong: FAILED)'} |")
    eff = efficiency(lines)
    if any(eff.values()):
        out += ["", "Scaling efficiency per reading, rate(N) / (N x rate(1)) of the SAME reading "
                "(the driver computes its own from `value`):", ""]
        out += ["| N | " + " | ".join(name for _, name in READINGS) + " |", "|---" * (len(READINGS) + 1) + "|"]
        for b in lines:
            n = b["n_gpus"]
            out.append(f"| {n} | " + " | ".join(fmt(eff[k].get(n)) for k, _ in READINGS) + " |")
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
    if any(b.get("rehearsal_note") for b in lines):
        out += ["", "Rehearsal lines (ranks sharing one GPU) are present: their rates are not N-GPU measurements."]
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
