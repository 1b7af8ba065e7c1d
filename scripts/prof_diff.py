"""Per-step kernel table from two rocprofv3 .db traces of the same program run with different
step counts (init + warmup kernels cancel out): (calls_b - calls_a) / (steps_b - steps_a).

    python scripts/prof_diff.py A.db STEPS_A B.db STEPS_B [top]
"""
import sqlite3
import sys
from collections import defaultdict


def load(path):
    cur = sqlite3.connect(path).cursor()
    q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    agg = defaultdict(lambda: [0, 0.0])
    for name, st, en in cur.execute(q):
        agg[name][0] += 1
        agg[name][1] += (en - st) / 1e6
    return agg


def main():
    a, na, b, nb = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    top = int(sys.argv[5]) if len(sys.argv) > 5 else 40
    A, Bd = load(a), load(b)
    k = nb - na
    rows = []
    for name in set(A) | set(Bd):
        ca, ta = A.get(name, (0, 0.0))
        cb, tb = Bd.get(name, (0, 0.0))
        rows.append((name, (cb - ca) / k, (tb - ta) / k))
    rows.sort(key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    print(f"per-step kernel time: {total:.2f} ms ({k} steps differenced)\n")
    print("| kernel | calls/step | ms/step | % | avg us |\n|---|---|---|---|---|")
    for name, c, t in rows[:top]:
        if abs(t) < 0.005:
            continue
        short = name if len(name) < 110 else name[:107] + "..."
        avg = 1000 * t / c if c > 0.5 else float("nan")
        print(f"| `{short}` | {c:.1f} | {t:.2f} | {100 * t / total:.1f} | {avg:.1f} |")


if __name__ == "__main__":
    main()
