"""The C-ABI library loads, exports every symbol include/gncde.h declares, and its struct layout matches
the ctypes mirror.  Host-only entry points (version, strerror, workspace sizing, path selection) are
exercised; nothing here launches a kernel."""
import ctypes
import os
import re
import subprocess

import pytest

from gncde import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gncde.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(gncde_\w+)\s*\(", txt, re.M)))


def test_header_declares_exactly_the_bound_symbols():
    assert declared_functions() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (gncde_\w+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing


def test_library_loads_and_reports_abi():
    lib = _lib.load()
    assert lib.gncde_abi_version() == _lib.ABI_VERSION
    assert lib.gncde_strerror(0) == b"ok"
    assert b"workspace" in lib.gncde_strerror(4)


def test_struct_layout_matches_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(f'''#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(GncdeProblem), offsetof(GncdeProblem, ts),
         offsetof(GncdeProblem, params), sizeof(GncdeSolver), offsetof(GncdeSolver, save_ts),
         offsetof(GncdeSolver, step_ts), offsetof(GncdeSolver, step_ts_len), offsetof(GncdeSolver, stage_rec),
         offsetof(GncdeSolver, stage_rec_len), offsetof(GncdeSolver, flags), offsetof(GncdeSolver, act_rec),
         offsetof(GncdeSolver, act_rec_len));
  return 0;
}}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", str(src), "-o", str(exe)], check=True)
    vals = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    P, S = _lib.GncdeProblem, _lib.GncdeSolver
    assert vals == [ctypes.sizeof(P), P.ts.offset, P.params.offset, ctypes.sizeof(S), S.save_ts.offset,
                    S.step_ts.offset, S.step_ts_len.offset, S.stage_rec.offset, S.stage_rec_len.offset,
                    S.flags.offset, S.act_rec.offset, S.act_rec_len.offset]


def _fake_problem(B=4, n=64, T=10, dims=(16, 16, 16, 16)):
    p = _lib.GncdeProblem()
    p.B, p.n, p.T, p.L = B, n, T, len(dims) - 1
    for i, d in enumerate(dims):
        p.dims[i] = d
    # host-only entry points only validate non-NULL-ness; nothing is dereferenced
    p.ts = p.coef = p.tcoef = p.fusion = p.params = 0x1000
    return p


def _fake_solver(method=_lib.RK4):
    s = _lib.GncdeSolver()
    s.method, s.controller, s.save_mode, s.grid_len = method, _lib.CTRL_GRID, _lib.SAVE_T1, 101
    s.grid = s.nsteps = 0x1000
    return s


def test_path_selection_and_workspace():
    lib = _lib.load()
    p, s = _fake_problem(), _fake_solver()
    buf = ctypes.create_string_buffer(64)
    assert lib.gncde_integrate_path(ctypes.byref(p), ctypes.byref(s), buf, 64) == 0
    assert buf.value == b"fused<64,16,3,rk4>"
    assert lib.gncde_workspace_bytes(ctypes.byref(p), ctypes.byref(s)) == 0  # fused path needs none
    assert lib.gncde_workspace_bytes(ctypes.byref(p), None) > 64 * 64 * 4 * 4 * 2
    p2 = _fake_problem(n=200)
    assert lib.gncde_integrate_path(ctypes.byref(p2), ctypes.byref(s), buf, 64) == 0
    assert buf.value == b"generic"
    assert lib.gncde_workspace_bytes(ctypes.byref(p2), ctypes.byref(s)) > 0
    s.flags = _lib.FLAG_GENERIC  # forced generic path: same problem, a workspace, both sweeps sized generic
    assert lib.gncde_integrate_path(ctypes.byref(p), ctypes.byref(s), buf, 64) == 0
    assert buf.value == b"generic"
    assert lib.gncde_workspace_bytes(ctypes.byref(p), ctypes.byref(s)) > 0
    s.flags = 4  # unknown flag bits are refused
    assert lib.gncde_integrate_path(ctypes.byref(p), ctypes.byref(s), buf, 64) == 1


@pytest.mark.parametrize("mutate,code", [
    (lambda p, s: setattr(p, "T", 1), 2),
    (lambda p, s: setattr(p, "L", 0), 2),
    (lambda p, s: setattr(p, "coef", None), 1),
    (lambda p, s: setattr(s, "method", 7), 1),
    (lambda p, s: setattr(s, "grid", None), 1),
])
def test_argument_validation_error_codes(mutate, code):
    lib = _lib.load()
    p, s = _fake_problem(), _fake_solver()
    mutate(p, s)
    buf = ctypes.create_string_buffer(64)
    assert lib.gncde_integrate_path(ctypes.byref(p), ctypes.byref(s), buf, 64) == code


def test_stage_record_floats():
    """gncde_stage_record_floats: (G-1)(S-1) n d_s for an fp32 GRID solve, else 0."""
    lib = _lib.load()
    p = _fake_problem()
    f = lambda p, s: lib.gncde_stage_record_floats(ctypes.byref(p), ctypes.byref(s))  # noqa: E731
    assert f(p, _fake_solver(_lib.RK4)) == 100 * 3 * 64 * 16
    assert f(p, _fake_solver(_lib.TSIT5)) == 100 * 5 * 64 * 16
    s = _fake_solver(_lib.TSIT5)
    s.controller, s.t0, s.t1, s.max_steps = _lib.CTRL_PID, 0x1000, 0x1000, 16
    assert f(p, s) == 0                                            # PID: replayed as a grid by the reverse mode
    assert f(_fake_problem(dims=(32, 32, 32)), _fake_solver()) == 100 * 3 * 64 * 32  # generic reverse sweep too
    assert f(_fake_problem(n=200), _fake_solver()) == 100 * 3 * 200 * 16
    bf = _fake_problem()
    bf.compute = _lib.COMPUTE_BF16
    assert f(bf, _fake_solver()) == 0                               # bf16 modes: the sweep recomputes stages
    bad = _fake_problem()
    bad.T = 1
    assert f(bad, _fake_solver()) == 0


def test_activation_record_floats():
    """gncde_activation_record_floats: (G-1) S (L-1) B n H where the fixed-grid forward takes the multi-kernel path
    and the reverse the per-layer kernels (BASELINE config 3's shape), else 0."""
    lib = _lib.load()
    f = lambda p, s: lib.gncde_activation_record_floats(ctypes.byref(p), ctypes.byref(s))  # noqa: E731
    cfg3 = _fake_problem(B=64, n=129, T=4, dims=(64, 64, 64, 1024))
    cfg3.cde_hidden, cfg3.cde_embed, cfg3.data_coef = 64, 8, 0x1000
    s = _fake_solver(_lib.TSIT5)
    s.grid_len = 31
    assert f(cfg3, s) == 30 * 6 * 2 * 64 * 129 * 64
    s.method = _lib.RK4
    assert f(cfg3, s) == 30 * 4 * 2 * 64 * 129 * 64
    assert f(_fake_problem(), _fake_solver()) == 0  # the fused forward / fused reverse sweep: no record
    pid = _fake_solver(_lib.TSIT5)
    pid.controller, pid.t0, pid.t1, pid.max_steps = _lib.CTRL_PID, 0x1000, 0x1000, 16
    assert f(cfg3, pid) == 0
    bf = _fake_problem(B=64, n=129, T=4, dims=(64, 64, 64, 1024))
    bf.cde_hidden, bf.cde_embed, bf.data_coef, bf.compute = 64, 8, 0x1000, _lib.COMPUTE_BF16
    assert f(bf, s) == 0


def test_stage_record_length_is_checked():
    """A stage record whose length is not gncde_stage_record_floats() is refused (GNCDE_ERR_ARG) by the forward
    (and, through the same validation, the reverse mode) instead of being written / read out of bounds."""
    lib = _lib.load()
    p, s = _fake_problem(), _fake_solver()
    buf = ctypes.create_string_buffer(64)
    s.stage_rec = 0x2000
    for length, code in ((100 * 3 * 64 * 16, 0), (100 * 3 * 64 * 16 - 1, 1), (0, 1)):
        s.stage_rec_len = length
        assert lib.gncde_integrate_path(ctypes.byref(p), ctypes.byref(s), buf, 64) == code, length
    bf = _fake_problem()
    bf.compute = _lib.COMPUTE_BF16  # no record exists for the bf16 modes
    s.stage_rec_len = 100 * 3 * 64 * 16
    assert lib.gncde_integrate_path(ctypes.byref(bf), ctypes.byref(s), buf, 64) == 1


def test_library_sha_matches_tree_sources():
    lib = _lib.load()
    assert lib.gncde_source_sha256().decode() == _lib.source_sha256()


def test_library_from_other_sources_is_refused(monkeypatch):
    """A library whose compiled-in source sha differs from this tree's is refused (build provenance)."""
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "source_sha256", lambda: "0" * 64)
    monkeypatch.delenv("GNCDE_LIB_UNVERIFIED", raising=False)
    with pytest.raises(_lib.GncdeError, match="built from kernel sources"):
        _lib.load()


def test_tampered_source_changes_the_tree_sha(tmp_path, monkeypatch):
    """The tree sha covers every kernel source byte: a one-byte edit of a copy of csrc/ gives another sha."""
    import shutil
    pkg = tmp_path / "pkg"
    shutil.copytree(os.path.join(_lib._PKG_ROOT, "csrc"), pkg / "csrc")
    (tmp_path / "include").mkdir()
    shutil.copy(HEADER, tmp_path / "include" / "gncde.h")
    monkeypatch.setattr(_lib, "_PKG_ROOT", str(pkg))
    base = _lib.source_sha256()
    assert base == _lib.load().gncde_source_sha256().decode()
    f = pkg / "csrc" / "gncde_rows.hip"
    f.write_bytes(f.read_bytes() + b" ")
    assert _lib.source_sha256() != base
