"""The C ABI library without a GPU: it loads, exports every entry point that
include/lfg.h declares, its struct layout matches the ctypes mirror, and
argument errors come back as codes.  No kernel is launched here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from lfit_python_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lfg.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lfg_[a-z_]+)\s*\(", text)))


def test_header_declares_and_library_exports_everything():
    names = declared_functions()
    assert "lfg_flux" in names and "lfg_lnprob" in names and len(names) >= 10
    L = _native.lib()
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_native.EXPORTS)
    nm = subprocess.run(["nm", "-D", "--defined-only", _native.LOAD_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r" T (lfg_[a-z_]+)", nm))
    assert set(names) <= exported


def test_tree_struct_layout_matches_ctypes(tmp_path):
    prog = tmp_path / "layout.c"
    prog.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "lfg.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(lfg_tree), offsetof(lfg_tree, gather),
         offsetof(lfg_tree, x), offsetof(lfg_tree, prior_norm), offsetof(lfg_tree, roche_priors),
         offsetof(lfg_tree, gp_gather), offsetof(lfg_tree, gp_ecl), offsetof(lfg_tree, fixed_invalid));
  return 0;
}''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(prog)], check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()))
    T = _native.LfgTree
    assert got == [ctypes.sizeof(T), T.gather.offset, T.x.offset, T.prior_norm.offset, T.roche_priors.offset,
                   T.gp_gather.offset, T.gp_ecl.offset, T.fixed_invalid.offset]


def test_constants_agree_with_header():
    text = open(HEADER).read()
    for name, val in (("LFG_NWD", _native.NWD), ("LFG_NDISC", _native.NDISC), ("LFG_NBS", _native.NBS),
                      ("LFG_NDONOR", _native.NDONOR), ("LFG_NGEO", _native.NGEO)):
        assert re.search(r"#define %s\s+%d\b" % (name, val), text), name


def test_argument_errors_without_gpu():
    L = _native.lib()
    assert L.lfg_workspace_size(0, 1) == 0
    ws1 = L.lfg_workspace_size(1024, 1)
    # symmetry-unique intervals (700 WD/disc + 100 spot, a and b) + unique donor tiles
    assert ws1 > 1024 * (2 * 800 + 5 * 100) * 8
    assert L.lfg_workspace_size(2048, 1) > ws1
    assert L.lfg_flux(None, 0, 18, None, None, 10, 1, None, None, None, None, 0, None) == -1
    assert L.lfg_flux(ctypes.c_void_p(8), 4, 15, None, None, 10, 1, None, None, None, None, 0, None) == -1
    # a valid call with too little workspace is refused before any launch
    assert L.lfg_flux(ctypes.c_void_p(8), 4, 18, ctypes.c_void_p(8), None, 10, 1, ctypes.c_void_p(8),
                      None, None, ctypes.c_void_p(8), 16, None) == -2
    assert L.lfg_lnprob(None, 4, None, None, None, None, 0, None) == -1
    assert L.lfg_stretch_propose(None, 15, 4, 0, 2.0, 1, 0, None, None, None) == -1
    assert L.lfg_roche(7, None, None, 1, None, None, None) == -1
    # a shard outside the half, an odd ensemble: refused before any launch
    vp8 = ctypes.c_void_p(8)
    assert L.lfg_stretch_step_shard(vp8, 64, 0, 2.0, 1, 0, 20, 16, vp8, vp8, None, vp8, vp8, 1 << 30, None,
                                    None) == -1
    assert L.lfg_stretch_accept_regen(vp8, vp8, 63, 4, 0, 2.0, 1, 0, vp8, None, None) == -1
    assert L.lfg_wdphases(None, None, None, 4, 10, None, None, None, None) == -1
    assert L.lfg_wdphases(None, None, None, 0, 10, None, None, None, None) == 0  # nothing to do
    assert L.lfg_gp_lnlike(None, None, None, 0, 10, None, None, 0, None, None) == -1
    assert L.lfg_version().startswith(b"lfg")


def test_layout_switch_without_gpu():
    """lfg_set_layout / lfg_layout (host-only): k_pair for one-tile S = 1
    trees by default, its LONG variant for sub-binned or longer chi^2
    eclipses, the two-kernel layout for long GP eclipses and when switched
    off; argument errors refused; the previous setting is returned and restored."""
    L = _native.lib()

    def tree(nsub, max_n, gp=0):  # lfg_layout reads the sizes only
        T = _native.LfgTree()
        T.E, T.ndim, T.nsub, T.max_n, T.gp = 1, 18, nsub, max_n, gp
        return ctypes.byref(T)

    assert L.lfg_layout(None) == -1
    assert L.lfg_set_layout(2) == -1 and L.lfg_set_layout(-3) == -1
    prev = L.lfg_set_layout(1)
    try:
        assert L.lfg_layout(tree(1, 300)) == 1
        assert L.lfg_layout(tree(1, 300, gp=1)) == 1   # GP trees: k_pair<true> for one tile
        assert L.lfg_layout(tree(5, 300)) == 2     # sub-binned: k_pair LONG
        assert L.lfg_layout(tree(1, 10000)) == 2   # more points than a tile: LONG
        assert L.lfg_layout(tree(1, 10000, gp=1)) == 0   # a long GP eclipse: two kernels
        assert b" layout=pair " in L.lfg_version()
        assert L.lfg_set_layout(0) == 1
        assert L.lfg_layout(tree(1, 300)) == 0
        assert L.lfg_layout(tree(5, 10000)) == 0
        assert b" layout=two_kernel " in L.lfg_version()   # the version names the layout in force
    finally:
        L.lfg_set_layout(prev)


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from lfit_python_amd import lfit, roche
    from tests.helpers import TRUTH18
    with pytest.raises(RuntimeError, match="GPU"):
        lfit.CV(TRUTH18).calcFlux(TRUTH18, np.linspace(-0.1, 0.1, 11))
    with pytest.raises(RuntimeError, match="GPU"):
        roche.xl1(0.1)


def test_rccl_unique_id_round_trip_keeps_nul_bytes():
    # the id travels as bytes through broadcast_object_list (comm.py); a NUL
    # inside it must not truncate it
    from lfit_python_amd import comm
    raw = bytes([7, 0, 9]) + bytes(range(125))
    uid = comm.uid_from(raw)
    assert comm.uid_bytes(uid) == raw
    with pytest.raises(ValueError):
        comm.uid_from(raw[:100])


def test_stale_library_is_rebuilt(tmp_path, monkeypatch):
    """build() decides by the compiled-in source hash, not file times: a
    library whose hash is not the tree's is rebuilt, the tree's is kept."""
    import shutil
    lib = tmp_path / "liblfg_hip.so"
    shutil.copy(_native.LIB_PATH, lib)
    h0 = _native.file_hash(str(lib))
    want = _native.source_hash()
    data = lib.read_bytes().replace(h0.encode(), want.encode())   # "the tree's" library
    lib.write_bytes(data.replace(want.encode(), b"0123456789abcdef"))   # a stale one
    assert _native.file_hash(str(lib)) == "0123456789abcdef"
    calls = []
    monkeypatch.setattr(_native, "LIB_PATH", str(lib))
    monkeypatch.setattr(_native.subprocess, "run", lambda cmd, check: (calls.append(cmd), shutil.copy(
        _native.LIB_PATH + ".orig", cmd[cmd.index("-o") + 1]))[0])
    (tmp_path / "liblfg_hip.so.orig").write_bytes(data)
    _native.build()
    # two hipcc runs: the split unit (k_pair's fold and LONG instantiations,
    # without machine LICM), then the library linked with it
    assert len(calls) == 2 and calls[0][-1] == _native.SPLIT_SOURCE and "-disable-machine-licm" in calls[0]
    assert ('-DLFG_SRC_HASH="%s"' % want) in calls[1] and "-disable-machine-licm" not in calls[1]
    assert _native.file_hash(str(lib)) == want
    assert not any(p.name.endswith(".tmp.o") for p in tmp_path.iterdir())
    _native.build()                      # now current: nothing rebuilt
    assert len(calls) == 2


def test_foreign_library_refused(tmp_path):
    """LFG_LIB without LFG_DIAGNOSTIC=1 is refused at import; with it, a
    library carrying another source hash fails verify() (what smoke() and the
    GPU test session run before any kernel)."""
    import shutil
    import sys
    foreign = tmp_path / "liblfg_foreign.so"
    h0 = _native.file_hash(_native.LIB_PATH)
    data = open(_native.LIB_PATH, "rb").read().replace(h0.encode(), b"fedcba9876543210")  # tag and lfg_version
    foreign.write_bytes(data)
    env = dict(os.environ, LFG_LIB=str(foreign))
    env.pop("LFG_DIAGNOSTIC", None)
    code = "import lfit_python_amd._native"
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "LFG_DIAGNOSTIC" in r.stderr
    env["LFG_DIAGNOSTIC"] = "1"
    code = ("import lfit_python_amd._native as n\n"
            "try:\n    n.verify()\nexcept RuntimeError as e:\n    print('refused', e)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True)
    assert "refused" in r.stdout and "fedcba9876543210" in r.stdout, r.stdout + r.stderr
    shutil.rmtree(tmp_path, ignore_errors=True)
