"""The library's Makefile rebuilds exactly what a header edit affects (round-5 advisor finding: an edit to
csrc/gncde_forms.h alone used to regenerate the provenance sha while relinking stale objects).

Dry runs (`make -n`) in a scratch copy of the package's Makefile, sources and dependency files, with the copied
objects' mtimes preserved: nothing is compiled and the real tree is not touched."""
import os
import re
import shutil
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "perm-equiv-graph-neural-cdes_amd")


def _compiled(tmp_pkg):
    out = subprocess.run(["make", "-n", "-C", tmp_pkg], capture_output=True, text=True, check=True).stdout
    return sorted(set(re.findall(r"-c csrc/(\w+)\.hip", out))), out


def _scratch(tmp_path, with_deps):
    pkg = tmp_path / "pkg"
    (tmp_path / "include").mkdir()
    shutil.copy2(os.path.join(ROOT, "include", "gncde.h"), tmp_path / "include" / "gncde.h")
    shutil.copytree(os.path.join(PKG, "csrc"), pkg / "csrc")
    shutil.copy2(os.path.join(PKG, "Makefile"), pkg / "Makefile")
    (pkg / "build").mkdir()
    (pkg / "gncde").mkdir()
    srcs = sorted(f[:-4] for f in os.listdir(pkg / "csrc") if f.endswith(".hip"))
    later = time.time() + 10
    for s in srcs:  # objects newer than every source: an up-to-date tree
        (pkg / "build" / f"{s}.o").write_bytes(b"")
        os.utime(pkg / "build" / f"{s}.o", (later, later))
        if with_deps:
            d = os.path.join(PKG, "build", f"{s}.d")
            if not os.path.exists(d):
                pytest.skip("the library has not been built with dependency files yet (make -C pkg)")
            shutil.copy2(d, pkg / "build" / f"{s}.d")
    for f in ("gncde_srcsha.c", "gncde_srcsha.o"):
        (pkg / "build" / f).write_bytes(b"")
        os.utime(pkg / "build" / f, (later, later))
    (pkg / "gncde" / "libgncde_hip.so").write_bytes(b"")
    os.utime(pkg / "gncde" / "libgncde_hip.so", (later + 1, later + 1))
    return str(pkg), srcs


def _touch(path, t):
    os.utime(path, (t, t))


def test_forms_header_edit_rebuilds_its_includers(tmp_path):
    pkg, srcs = _scratch(tmp_path, with_deps=True)
    assert _compiled(pkg)[0] == []
    _touch(os.path.join(pkg, "csrc", "gncde_forms.h"), time.time() + 100)
    built, out = _compiled(pkg)
    includers = sorted(s for s in srcs
                       if '#include "gncde_forms.h"' in open(os.path.join(pkg, "csrc", s + ".hip")).read())
    assert includers and built == includers, (built, includers)
    assert "gncde_generic" in built and "gncde_layer" in built
    assert "libgncde_hip.so" in out and "gncde_source_sha256" in out  # relinked with a regenerated sha


def test_internal_header_edit_rebuilds_everything(tmp_path):
    pkg, srcs = _scratch(tmp_path, with_deps=True)
    _touch(os.path.join(pkg, "csrc", "gncde_internal.h"), time.time() + 100)
    assert _compiled(pkg)[0] == srcs


def test_objects_without_dependency_files_depend_on_every_header(tmp_path):
    pkg, srcs = _scratch(tmp_path, with_deps=False)
    assert _compiled(pkg)[0] == []
    _touch(os.path.join(pkg, "csrc", "gncde_forms.h"), time.time() + 100)
    assert _compiled(pkg)[0] == srcs
