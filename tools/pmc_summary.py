#!/usr/bin/env python3
"""Summarise rocprofv3 outputs for the dominant kernel.

  tools/pmc_summary.py stats  gpurun_out/prof/run_kernel_stats.csv            -> top kernels table
  tools/pmc_summary.py traffic gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE WORKLOAD KERNEL OUT.json
  tools/pmc_summary.py counters DIR...                                          -> mean per kernel/counter

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are collected in
separate passes (TCC slots), are in KiB, and on gfx950 FETCH_SIZE reports half the bytes of a wide
(16 B/lane) coalesced read, so  hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def counters(dirs, match="k_fused"):
    acc = defaultdict(list)
    for d in dirs:
        for r in _rows(d):
            if match and match not in r["Kernel_Name"]:
                continue
            acc[(r["Kernel_Name"][:90], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    mode = sys.argv[1]
    if mode == "stats":
        with open(sys.argv[2]) as fh:
            rows = list(csv.DictReader(fh))
        for r in rows[:8]:
            print(f'{float(r["Percentage"]):6.2f}%  calls={r["Calls"]:>5}  avg={float(r["AverageNs"]) / 1e3:10.1f} us  '
                  f'{r["Name"][:100]}')
    elif mode == "counters":
        for (k, c), v in sorted(counters(sys.argv[2:], os.environ.get("MATCH", "k_fused")).items()):
            print(f"{c:32s} {v:16.1f}  {k}")
    elif mode == "table":  # one line per kernel over tools/pmc_configs.sh's pass directories (all kernels)
        acc = defaultdict(lambda: defaultdict(list))
        for d in sys.argv[2:]:
            for r in _rows(d):
                acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        g = lambda c, k: (sum(c[k]) / len(c[k])) if c.get(k) else 0.0  # noqa: E731
        rows = []
        for name, c in acc.items():
            waves = g(c, "SQ_WAVES")
            pw = lambda k: g(c, k) / waves if waves else 0.0  # noqa: E731
            hbm = (2.0 * g(c, "FETCH_SIZE") + g(c, "WRITE_SIZE")) * 1024.0
            short = name.replace("gncde::(anonymous namespace)::", "").replace("void ", "")[:60]
            if "gncde" not in name:
                continue
            rows.append((hbm, f"{short:60s} dispatches={len(c.get('SQ_WAVES', [])):5d} waves={waves:8.0f} "
                              f"VALU/wave={pw('SQ_INSTS_VALU'):8.1f} MFMA/wave={pw('SQ_INSTS_VALU_MFMA_F32'):6.1f} "
                              f"LDS/wave={pw('SQ_INSTS_LDS'):6.1f} bank_conflict_cyc={g(c, 'SQ_LDS_BANK_CONFLICT'):10.0f} "
                              f"mfma_busy={g(c, 'SQ_VALU_MFMA_BUSY_CYCLES'):10.0f} wait_any_per_wave={pw('SQ_WAIT_ANY'):9.0f} "
                              f"busy_cyc={g(c, 'SQ_BUSY_CYCLES'):9.0f} hbm_bytes={hbm:12.0f} "
                              f"fetch_kib={g(c, 'FETCH_SIZE'):9.1f} write_kib={g(c, 'WRITE_SIZE'):9.1f}"))
        for _, line in sorted(rows, key=lambda x: -x[0]):
            print(line)
    elif mode == "traffic":
        fetch_dir, write_dir, workload, kernel, out = sys.argv[2:7]
        f = counters([fetch_dir]).items()
        w = counters([write_dir]).items()
        fetch = [v for (k, c), v in f if c == "FETCH_SIZE"]
        write = [v for (k, c), v in w if c == "WRITE_SIZE"]
        if not fetch or not write:
            raise SystemExit("no FETCH_SIZE/WRITE_SIZE rows for the fused kernel")
        fkb, wkb = fetch[0], write[0]
        import hashlib
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        src = os.path.join(root, "perm-equiv-graph-neural-cdes_amd", "csrc", "gncde_fused.hip")
        with open(src, "rb") as fh:
            sha = hashlib.sha256(fh.read()).hexdigest()[:16]
        d = {"workload": workload, "kernel": kernel, "source_sha16": sha, "fetch_size_kib": fkb, "write_size_kib": wkb,
             "hbm_bytes_per_launch": (2.0 * fkb + wkb) * 1024.0,
             "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md §HBM)"}
        with open(out, "w") as fh:
            json.dump(d, fh, indent=1)
        print(json.dumps(d))


if __name__ == "__main__":
    main()
