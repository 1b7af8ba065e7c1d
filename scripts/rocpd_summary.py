"""Summarise a rocprofv3 .db (rocpd schema) into per-kernel stats (markdown table)."""
import sqlite3
import sys
from collections import defaultdict


def summarize(path, top=40):
    db = sqlite3.connect(path)
    cur = db.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(rocpd_kernel_dispatch)")]
    q = ("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    agg = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for name, st, en in cur.execute(q):
        dur = (en - st) / 1e6
        agg[name][0] += 1
        agg[name][1] += dur
        total += dur
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    out = [f"total kernel time: {total:.1f} ms over {sum(v[0] for v in agg.values())} dispatches", "",
           "| kernel | calls | total ms | % | avg us |", "|---|---|---|---|---|"]
    for name, (n, t) in rows[:top]:
        short = name if len(name) < 110 else name[:107] + "..."
        out.append(f"| `{short}` | {n} | {t:.2f} | {100*t/total:.1f} | {1000*t/n:.1f} |")
    return "\n".join(out)


if __name__ == "__main__":
    print(summarize(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40))
