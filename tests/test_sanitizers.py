"""SURVEY §5 "Race detection / sanitizers": the C restatement of the oracle under AddressSanitizer + UBSan.

`make -C oracle asan` builds oracle/build/libgncde_oracle_asan.so from the same gncde_oracle.c.  The checks run in a
child process whose environment alone preloads libasan (the sanitizer runtime must come first in the library list;
nothing here changes this process's environment):
  * tests/test_c_oracle.py passes against the sanitized build (every finding is fatal: -fno-sanitize-recover=all);
  * a deliberately out-of-range call (a step count one past its grid row) is caught, which shows the build under
    test is the instrumented one.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
ASAN_LIB = os.path.join(ORACLE, "build", "libgncde_oracle_asan.so")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True, check=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def asan_env():
    if os.environ.get("LD_PRELOAD"):
        pytest.skip("a preload is already set in this environment; the sanitizer runtime cannot come first")
    libasan = _runtime("libasan.so")
    if libasan is None:
        pytest.skip("gcc has no libasan runtime")
    subprocess.run(["make", "-C", ORACLE, "-s", "asan"], check=True)
    env = dict(os.environ)
    env.update(LD_PRELOAD=libasan, GNCDE_ORACLE_LIB=ASAN_LIB,
               # CPython's own allocations are reported as leaks at interpreter exit; memory errors stay fatal.
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24",
               OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    return env


def test_c_oracle_suite_under_asan_ubsan(asan_env):
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_c_oracle.py")],
                       cwd=ROOT, env=asan_env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "1 passed" in out, out[-2000:]


_OVERRUN = r"""
import numpy as np
from oracle import c_oracle
from tests.golden import make_golden as MG
assert c_oracle.LIB.endswith("libgncde_oracle_asan.so"), c_oracle.LIB
z = np.load("tests/golden/rk4_undirected_n10_L3.npz")
params = MG.load_layers(z)
coef = np.stack([z["d"][..., 1], z["c"][..., 1], z["b"][..., 1], z["a"][..., 1]], axis=2)
tcoef = np.stack([z["d"][..., 0].mean(-2), z["c"][..., 0].mean(-2), z["b"][..., 0].mean(-2)], axis=2)
B = z["grid"].shape[0]
G = 400                                    # > 1 KB per row: a plain malloc'd buffer, redzone right after it
grid = np.zeros((B, G), np.float32)
grid[:, :z["grid"].shape[1]] = z["grid"]
nsteps = np.array(z["nsteps"], np.int32)
nsteps[-1] = G                             # reads grid[B-1, G]: one element past the array
c_oracle.rk4(z["ts"], coef, tcoef, params.layers, grid, nsteps, z["y0"], nthreads=1)
print("NOT CAUGHT")
"""


def test_asan_build_catches_an_overrun(asan_env):
    r = subprocess.run([sys.executable, "-c", _OVERRUN], cwd=ROOT, env=asan_env, capture_output=True, text=True,
                       timeout=600)
    out = r.stdout + r.stderr
    assert "NOT CAUGHT" not in out, out[-3000:]
    assert r.returncode == 23 and "heap-buffer-overflow" in out, (r.returncode, out[-3000:])
