"""Per-stream busy time and the main-stream critical path of a training step, from one
rocprofv3 ``--kernel-trace`` database (rocpd sqlite).

Why: a per-kernel table that sums every dispatch (scripts/prof_diff.py) adds up kernels that ran
CONCURRENTLY on side streams (the DDP grad-norm stream, RCCL), so its total is not the step time and
a kernel that looks expensive there may cost the critical path nothing. This tool:

  * finds step boundaries by a marker kernel that runs once per step on the main (compute)
    stream (default: the fused AdamW, ``adamw``), and takes the window of the LAST ``--steps``
    steps (init and warmup fall outside it);
  * for every HIP stream: dispatches, summed kernel time and busy time (union of its kernels'
    intervals) inside the window;
  * for the main stream (the marker's stream): busy time + idle gaps = the window, i.e. the
    critical path; gaps are split into "covered" (another stream was busy) and "device idle";
  * a per-kernel table of MAIN-stream time only (sums to the main stream's busy time), plus the
    side streams' kernels, and how much of the side-stream time overlapped main-stream kernels.

    python scripts/critical_path.py TRACE.db --steps 3 [--marker adamw] [--top 30] > profiles/X_cp.md
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def load(path):
    cur = sqlite3.connect(path).cursor()
    q = ("select s.kernel_name, d.stream_id, d.queue_id, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    return [(n, int(sid), int(qid), int(a), int(b)) for n, sid, qid, a, b in cur.execute(q)]


def union_len(iv):
    """Total length of the union of [a, b) intervals (sorted by a)."""
    tot, cur_a, cur_b = 0, None, None
    for a, b in sorted(iv):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def merge(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def intersect_len(xs, ys):
    """Length of the intersection of two merged interval lists."""
    i = j = 0
    tot = 0
    while i < len(xs) and j < len(ys):
        a = max(xs[i][0], ys[j][0])
        b = min(xs[i][1], ys[j][1])
        if b > a:
            tot += b - a
        if xs[i][1] < ys[j][1]:
            i += 1
        else:
            j += 1
    return tot


def short(name, n=100):
    return name if len(name) <= n else name[: n - 3] + "..."


def analyse(rows, steps, marker):
    marks = [r for r in rows if marker in r[0]]
    if len(marks) < steps + 1:
        raise SystemExit(f"need >= {steps + 1} '{marker}' dispatches to bound {steps} steps, found {len(marks)}")
    main_sid = marks[-1][1]
    t0, t1 = marks[-steps - 1][4], marks[-1][4]  # end of the marker before the window .. end of the last
    win = [(n, s, q, max(a, t0), min(b, t1)) for n, s, q, a, b in rows if b > t0 and a < t1]
    by_stream = defaultdict(list)
    for n, s, q, a, b in win:
        by_stream[s].append((n, a, b))
    span = t1 - t0
    main_iv = merge([(a, b) for _, a, b in by_stream[main_sid]])
    main_busy = sum(b - a for a, b in main_iv)
    others = merge([(a, b) for s, ks in by_stream.items() if s != main_sid for _, a, b in ks])
    gaps = []
    prev = t0
    for a, b in main_iv:
        if a > prev:
            gaps.append([prev, a])
        prev = max(prev, b)
    if t1 > prev:
        gaps.append([prev, t1])
    gap_total = sum(b - a for a, b in gaps)
    gap_covered = intersect_len(gaps, others)
    out = []
    ms = lambda ns: ns / 1e6 / steps  # noqa: E731 -- ns over the window -> ms per step
    out.append(f"# Critical path over the last {steps} steps (marker `{marker}`, main stream {main_sid})\n")
    out.append("| quantity | ms/step |\n|---|---|")
    out.append(f"| window (wall, marker to marker) | {ms(span):.2f} |")
    out.append(f"| main stream busy (union of its kernels) | {ms(main_busy):.2f} |")
    out.append(f"| main stream gaps | {ms(gap_total):.2f} |")
    out.append(f"| -- of which another stream was busy | {ms(gap_covered):.2f} |")
    out.append(f"| -- of which the device was idle | {ms(gap_total - gap_covered):.2f} |")
    out.append(f"| side-stream busy overlapping main-stream kernels | {ms(intersect_len(main_iv, others)):.2f} |")
    out.append("")
    out.append("## Streams\n\n| stream | dispatches/step | kernel ms/step (sum) | busy ms/step (union) |\n|---|---|---|---|")
    for s, ks in sorted(by_stream.items(), key=lambda kv: -len(kv[1])):
        tag = " (main)" if s == main_sid else ""
        out.append(f"| {s}{tag} | {len(ks) / steps:.1f} | {ms(sum(b - a for _, a, b in ks)):.2f} | "
                   f"{ms(union_len([(a, b) for _, a, b in ks])):.2f} |")
    out.append("")
    out.append("## Main-stream kernels (sums to the main stream's busy time)\n")
    out.append("| kernel | calls/step | ms/step | % of window |\n|---|---|---|---|")
    agg = defaultdict(lambda: [0, 0])
    for n, a, b in by_stream[main_sid]:
        agg[n][0] += 1
        agg[n][1] += b - a
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:TOP[0]]:
        out.append(f"| `{short(n)}` | {c / steps:.1f} | {ms(t):.2f} | {100.0 * t / span:.1f} |")
    side = defaultdict(lambda: [0, 0])
    for s, ks in by_stream.items():
        if s == main_sid:
            continue
        for n, a, b in ks:
            side[n][0] += 1
            side[n][1] += b - a
    if side:
        out.append("\n## Side-stream kernels (off the critical path unless the main stream waits on them)\n")
        out.append("| kernel | calls/step | ms/step |\n|---|---|---|")
        for n, (c, t) in sorted(side.items(), key=lambda kv: -kv[1][1])[:TOP[0]]:
            out.append(f"| `{short(n)}` | {c / steps:.1f} | {ms(t):.2f} |")
    return "\n".join(out) + "\n", ms(span)


TOP = [30]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--wall-ms", type=float, default=None,
                    help="un-profiled ms/step to compare the critical path against")
    a = ap.parse_args()
    TOP[0] = a.top
    text, cp = analyse(load(a.db), a.steps, a.marker)
    print(text)
    if a.wall_ms:
        print(f"critical path {cp:.2f} ms/step vs un-profiled {a.wall_ms:.2f} ms/step: "
              f"{100.0 * (cp - a.wall_ms) / a.wall_ms:+.1f} %")


if __name__ == "__main__":
    main()
