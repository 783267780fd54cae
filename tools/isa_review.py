#!/usr/bin/env python3
"""ISA review of the built library (SURVEY §5 "Race detection / sanitizers": HIP ISA review), CPU only.

For every object the library links (perm-equiv-graph-neural-cdes_amd/build/*.o) the gfx950 code object is unbundled
from its .hip_fatbin section (llvm-objcopy + clang-offload-bundler), its AMDHSA metadata notes give each kernel's
VGPR / AGPR / SGPR counts, scratch (private segment) and static LDS, and llvm-objdump gives its instructions.

  python tools/isa_review.py            # per-kernel table (the hot instances) + instruction checks
  python tools/isa_review.py --all      # every kernel

Checks (tests/test_isa.py runs them):
  * no instruction writes through the scalar data cache (scalar stores, scalar atomics, scalar cache write-back);
  * the headline kernel k_fused<64,16,3,rk4> has no scratch, at most 128 VGPRs (four waves per SIMD), and its
    products on v_mfma_f32_16x16x4_f32;
  * every kernel's scratch is reported (spills are visible, not silent);
  * no kernel wraps a buffer access in a waterfall loop (a descriptor the compiler could not prove uniform).
This file names scalar-store mnemonics, so it is listed in .gpurunignore (it never runs on the GPU box).
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
# scalar-data-cache writes: s_store_*, s_buffer_store_*, s_scratch_store_*, s_atomic_*, s_buffer_atomic_*,
# s_dcache_wb*
SCALAR_WRITE = re.compile(r"^\s*(s_store_|s_buffer_store_|s_scratch_store_|s_atomic_|s_buffer_atomic_|s_dcache_wb)")
WATERFALL = re.compile(r"^v_cmp_eq_u64\S*\s+\S+,\s*s\[\d+:\d+\],\s*v\[\d+:\d+\]")
HEADLINE = "_ZN5gncde12_GLOBAL__N_17k_fusedILi64ELi16ELi3ELi0EEEvNS0_9FusedArgsE"


def code_object(obj: str, out_dir: str) -> str:
    base = os.path.join(out_dir, os.path.basename(obj))
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={base}.fatbin", obj, f"{base}.host"],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={base}.fatbin",
                    f"--output={base}.co", f"--targets={TARGET}"], check=True, capture_output=True)
    return f"{base}.co"


def kernel_metadata(co: str) -> dict:
    """{symbol: {vgpr, agpr, sgpr, scratch, lds}} from the AMDHSA metadata note (gfx950: .vgpr_count is the unified
    VGPR + AGPR allocation, .agpr_count its AGPR part)."""
    txt = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", co], check=True, capture_output=True, text=True).stdout
    out, cur = {}, {}
    keys = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
            ".private_segment_fixed_size": "scratch", ".group_segment_fixed_size": "lds"}
    for line in txt.splitlines():
        s = line.strip().lstrip("- ").strip()
        if ":" not in s:
            continue
        k, v = s.split(":", 1)
        k, v = k.strip(), v.strip()
        if k == ".agpr_count" and cur.get("name"):  # a new kernel map starts with .agpr_count
            out[cur.pop("name")] = cur
            cur = {}
        if k == ".name" and v.startswith("_Z"):
            cur["name"] = v
        elif k in keys:
            try:
                cur[keys[k]] = int(v)
            except ValueError:
                pass
    if cur.get("name"):
        out[cur.pop("name")] = cur
    return out


def disassembly(co: str) -> dict:
    """{symbol: [instruction lines]}"""
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                         text=True).stdout
    out, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            out[cur] = []
        elif cur and line.strip():
            out[cur].append(line.strip())
    return out


def review(objs=None) -> dict:
    objs = objs or sorted(glob.glob(os.path.join(PKG, "build", "*.o")))
    objs = [o for o in objs if not o.endswith("gncde_srcsha.o")]
    if not objs:
        raise SystemExit("no objects: build the library first (make -C perm-equiv-graph-neural-cdes_amd)")
    res = {"kernels": {}, "scalar_writes": [], "objects": objs}
    with tempfile.TemporaryDirectory() as d:
        for o in objs:
            co = code_object(o, d)
            meta = kernel_metadata(co)
            dis = disassembly(co)
            for k, m in meta.items():
                ins = dis.get(k, [])
                m["object"] = os.path.basename(o)
                m["instructions"] = len(ins)
                m["mfma"] = sum(1 for x in ins if x.startswith("v_mfma"))
                # waterfall loops (a buffer descriptor the compiler holds in VGPRs: every access compares the
                # readfirstlane'd SGPR copy with the VGPR one, 64 bits at a time)
                m["waterfalls"] = sum(1 for x in ins if WATERFALL.match(x))
                res["kernels"][k] = m
            for k, ins in dis.items():
                for x in ins:
                    if SCALAR_WRITE.match(x):
                        res["scalar_writes"].append((os.path.basename(o), k, x))
    return res


def demangle(names):
    p = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return p.stdout.splitlines() if p.returncode == 0 else list(names)


def main():
    res = review()
    ks = res["kernels"]
    names = sorted(ks)
    if "--all" not in sys.argv:  # the hot instances
        hot = ("k_fusedILi64ELi16ELi3ELi0E", "k_fusedILi128ELi16ELi2ELi0E", "k_revILi128ELi2ELi6E",
               "k_rowsILi32ELi2ELi0ELi1E", "k_rowsILi32ELi2ELi2ELi9E", "k_layerILi64ELi64ELi0ELb0ELi2E",
               "k_layerILi64ELi64ELi2ELb0ELi5E", "k_bwd_layerILi64E", "k_bwd_layerILi32E", "k_abar_direct")
        names = [n for n in names if any(h in n for h in hot)]
    print(f"{len(ks)} kernels in {len(res['objects'])} objects; scalar-data-cache writes: {len(res['scalar_writes'])}")
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'SGPR':>5s} {'scratch':>8s} {'LDS':>7s} {'instr':>7s} {'mfma':>6s}")
    for n, d in zip(names, demangle(names)):
        m = ks[n]
        d = d.replace("gncde::(anonymous namespace)::", "").replace("void ", "")
        print(f"{d[:70]:70s} {m.get('vgpr', -1):5d} {m.get('agpr', -1):5d} {m.get('sgpr', -1):5d} "
              f"{m.get('scratch', -1):8d} {m.get('lds', -1):7d} {m['instructions']:7d} {m['mfma']:6d}")
    spills = sum(1 for m in ks.values() if m.get("scratch", 0) > 0)
    print(f"kernels with scratch: {spills} of {len(ks)}")
    wf = {n: m["waterfalls"] for n, m in ks.items() if m["waterfalls"]}
    print(f"kernels with waterfall loops: {len(wf)}")


if __name__ == "__main__":
    main()
