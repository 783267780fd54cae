"""Summarise a rocprofv3 rocpd database (--kernel-trace): per-kernel totals inside a time window, the kernels'
busy time and the window's wall span (busy/wall < 1 = launch gaps).  Windows are split at gaps longer than
--gap-ms (e.g. between the configs of tools/bench_configs.py)."""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--gap-ms", type=float, default=50.0)
    ap.add_argument("--top", type=int, default=14)
    ap.add_argument("--min-kernels", type=int, default=200)
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    rows = list(con.execute("select name, start, end from kernels order by start"))
    wins, cur = [], []
    for r in rows:
        if cur and r[1] - cur[-1][2] > args.gap_ms * 1e6:
            wins.append(cur)
            cur = []
        cur.append(r)
    if cur:
        wins.append(cur)
    for w in wins:
        if len(w) < args.min_kernels:
            continue
        agg = defaultdict(lambda: [0, 0.0])
        busy = 0.0
        for name, s, e in w:
            a = agg[name.replace("(anonymous namespace)::", "").split("(")[0][-60:]]
            a[0] += 1
            a[1] += (e - s) / 1e3
            busy += (e - s) / 1e3
        wall = (w[-1][2] - w[0][1]) / 1e3
        print(f"--- window: {len(w)} kernels, wall {wall / 1e3:.2f} ms, busy {busy / 1e3:.2f} ms ({busy / wall:.0%})")
        for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[: args.top]:
            print(f"  {t / 1e3:9.2f} ms {c:7d} x {t / c:8.2f} us  {k}")


if __name__ == "__main__":
    main()
