"""Loader for liblfg_hip.so, the gfx950 HIP library behind include/lfg.h.

The product path has no CPU fallback: every public entry point of this
package goes through the HIP kernels, and fails loudly when the library or a
GPU is missing.
"""
import ctypes
import hashlib
import os
import re
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(_HERE)
LIB_DIR = os.path.join(_HERE, "_lib")
LIB_PATH = os.path.join(LIB_DIR, "liblfg_hip.so")
# diagnostic builds (e.g. -DLFG_PROFILE_SETUP) are loaded through LFG_LIB,
# and only with LFG_DIAGNOSTIC=1 set as well: a stray LFG_LIB must not swap
# the product library silently
LOAD_PATH = LIB_PATH
if os.environ.get("LFG_LIB"):
    if os.environ.get("LFG_DIAGNOSTIC") != "1":
        raise RuntimeError("LFG_LIB=%s is set without LFG_DIAGNOSTIC=1: diagnostic builds are loaded only on "
                           "request (unset LFG_LIB to load %s)" % (os.environ["LFG_LIB"], LIB_PATH))
    LOAD_PATH = os.environ["LFG_LIB"]
SOURCES = [os.path.join(_HERE, "csrc", "lfg.hip"), os.path.join(_HERE, "csrc", "lfg_components.hip")]
# k_pair's fold and LONG instantiations: lfg.hip again, compiled on its own
# without machine LICM (the reason: lfg.hip, lfg_pair_launch_split)
SPLIT_SOURCE = os.path.join(_HERE, "csrc", "lfg_pair_split.hip")
SPLIT_FLAGS = ["-mllvm", "-disable-machine-licm"]
HEADERS = [os.path.join(_HERE, "csrc", "lfg_device.hpp"),
           os.path.join(_HERE, "csrc", "lfg_tables.hpp"),
           os.path.join(_HERE, "csrc", "lfg_stream_table.h"),
           os.path.join(REPO, "include", "lfg.h")]
INCLUDE = os.path.join(REPO, "include")
ARCH = "gfx950"

# element grid (MODEL_SPEC.md section 5; mirrors include/lfg.h)
NWD, NDISC, NBS, NDONOR = 400, 1000, 100, 400
NEL = NWD + NDISC + NBS
NGEO = 48

STATUS_TEXT = {
    0: "ok",
    1: "invalid mass ratio q",
    2: "dphi has no inclination solution (dphi >= findphi(q, 90) or <= 0)",
    3: "invalid geometry (rwd, rdisc, scale or bright-spot exponents)",
    4: "the gas stream does not reach the disc radius",
    5: "non-finite or wrong-length parameter vector",
}


class LfgTree(ctypes.Structure):
    """ctypes mirror of struct lfg_tree (include/lfg.h)."""
    _fields_ = [
        ("E", ctypes.c_int), ("ndim", ctypes.c_int), ("nsub", ctypes.c_int),
        ("max_n", ctypes.c_int),
        ("gather", ctypes.c_void_p), ("npars", ctypes.c_void_p),
        ("consts", ctypes.c_void_p), ("off", ctypes.c_void_p),
        ("x", ctypes.c_void_p), ("y", ctypes.c_void_p),
        ("ye", ctypes.c_void_p), ("w", ctypes.c_void_p),
        ("prior_type", ctypes.c_void_p), ("prior_p1", ctypes.c_void_p),
        ("prior_p2", ctypes.c_void_p), ("prior_norm", ctypes.c_void_p),
        ("roche_priors", ctypes.c_int),
        ("gp", ctypes.c_int),
        ("gp_gather", ctypes.c_void_p), ("gp_base", ctypes.c_void_p),
        ("gp_ecl", ctypes.c_void_p),
        ("fixed_invalid", ctypes.c_int),
        ("prior_c", ctypes.c_void_p),
    ]


EXPORTS = ("lfg_workspace_size", "lfg_workspace_size_tree", "lfg_flux", "lfg_lnlike", "lfg_lnprob", "lfg_lnprior", "lfg_lnprob_timed",
           "lfg_stretch_lnprob_accept", "lfg_stretch_step_half", "lfg_stretch_step_half_spec",
           "lfg_stretch_step_shard", "lfg_stretch_step_shard_spec", "lfg_stretch_accept_regen_spec",
           "lfg_stretch_accept_regen", "lfg_stretch_step_shard_fold", "lfg_stretch_apply_verdicts",
           "lfg_elements", "lfg_roche", "lfg_stretch_propose", "lfg_stretch_accept",
           "lfg_stretch_propose_dev", "lfg_stretch_accept_dev", "lfg_event_create", "lfg_event_destroy",
           "lfg_event_elapsed_ms", "lfg_wdphases", "lfg_gp_lnlike", "lfg_component_workspace_size",
           "lfg_component", "lfg_version", "lfg_layout", "lfg_set_layout")


FLAGS = ["--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-shared"]
HASH_TAG = b"lfg-src-hash:"


def source_hash():
    """16 hex digits of SHA-256 over the library's sources, headers and
    compile flags: compiled into the library (lfg_version, and a tag string
    build() reads back), so a stale or foreign binary is told apart from
    the one this tree builds."""
    h = hashlib.sha256()
    for p in SOURCES + [SPLIT_SOURCE] + HEADERS:
        h.update(os.path.relpath(p, REPO).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS + SPLIT_FLAGS).encode())
    return h.hexdigest()[:16]


def file_hash(path):
    """the source hash compiled into the library at `path` (None: no tag)"""
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    m = re.search(re.escape(HASH_TAG) + rb"([0-9a-f]{16})", data)
    return m.group(1).decode() if m else None


def needs_build():
    return file_hash(LIB_PATH) != source_hash()


def build(force=False, verbose=False):
    """Compile liblfg_hip.so in-tree for gfx950 (hipcc cross-compiles
    offline) unless the library there was built from exactly these sources
    and flags (its compiled-in source hash, not file times, decides)."""
    os.makedirs(LIB_DIR, exist_ok=True)
    want = source_hash()
    if not force and file_hash(LIB_PATH) == want:
        return LIB_PATH
    tmp = LIB_PATH + ".tmp"
    obj = LIB_PATH + ".split.tmp.o"
    cmds = [["hipcc"] + [f for f in FLAGS if f != "-shared"] + SPLIT_FLAGS + ["-I", INCLUDE, "-c", "-o", obj,
                                                                            SPLIT_SOURCE],
            ["hipcc"] + FLAGS + ['-DLFG_SRC_HASH="%s"' % want, "-I", INCLUDE, "-o", tmp] + SOURCES + ["-x", "none", obj]]
    try:
        for cmd in cmds:
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
    finally:
        if os.path.exists(obj):
            os.remove(obj)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


def loaded_hash():
    """the source hash of the library this process loaded (lfg_version's src=)"""
    v = lib().lfg_version().decode()
    m = re.search(r"src=([0-9a-f]{16}|unhashed)", v)
    return m.group(1) if m else None


def verify():
    """Raise unless the loaded library is the one this tree's sources build
    (smoke() and the GPU test session check it before any kernel runs)."""
    got, want = loaded_hash(), source_hash()
    if got != want:
        raise RuntimeError("loaded %s carries source hash %s, the tree's sources hash to %s: a stale or foreign "
                           "library (rebuild with __graft_entry__.build())" % (LOAD_PATH, got, want))
    return got


_lib = None
_lock = threading.Lock()


def lib():
    """The loaded library; raises if it was never built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LOAD_PATH):
            raise RuntimeError(
                "liblfg_hip.so is missing (%s): run __graft_entry__.build() or "
                "lfit_python_amd._native.build(); there is no CPU fallback" % LOAD_PATH)
        L = ctypes.CDLL(LOAD_PATH)
        vp, ip, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.lfg_workspace_size.restype = sz
        L.lfg_workspace_size.argtypes = [ip, ip]
        L.lfg_workspace_size_tree.restype = sz
        L.lfg_workspace_size_tree.argtypes = [ip, ctypes.POINTER(LfgTree)]
        L.lfg_flux.restype = ip
        L.lfg_flux.argtypes = [vp, ip, ip, vp, vp, ip, ip, vp, vp, vp, vp, sz, vp]
        L.lfg_lnlike.restype = ip
        L.lfg_lnlike.argtypes = [vp, ip, ip, vp, vp, ip, ip, vp, vp, vp, vp, vp, sz, vp]
        L.lfg_lnprob.restype = ip
        L.lfg_lnprob.argtypes = [vp, ip, ctypes.POINTER(LfgTree), vp, vp, vp, sz, vp]
        L.lfg_lnprior.restype = ip
        L.lfg_lnprior.argtypes = [vp, ip, ctypes.POINTER(LfgTree), vp, vp, sz, vp]
        L.lfg_elements.restype = ip
        L.lfg_elements.argtypes = [vp, ip, ip, vp, vp, vp, vp, vp, vp, vp, sz, vp]
        L.lfg_roche.restype = ip
        L.lfg_roche.argtypes = [ip, vp, vp, ip, vp, vp, vp]
        L.lfg_lnprob_timed.restype = ip
        L.lfg_lnprob_timed.argtypes = [vp, ip, ctypes.POINTER(LfgTree), vp, vp, vp, sz, vp,
                                       ctypes.POINTER(vp)]
        u64, f64 = ctypes.c_ulonglong, ctypes.c_double
        L.lfg_stretch_propose.restype = ip
        L.lfg_stretch_propose.argtypes = [vp, ip, ip, ip, f64, u64, u64, vp, vp, vp]
        L.lfg_stretch_accept.restype = ip
        L.lfg_stretch_accept.argtypes = [vp, vp, ip, ip, ip, vp, vp, vp, u64, u64, vp, vp]
        L.lfg_stretch_lnprob_accept.restype = ip
        L.lfg_stretch_lnprob_accept.argtypes = [vp, vp, ip, ip, vp, vp, ctypes.POINTER(LfgTree), u64, u64, vp,
                                                vp, vp, sz, vp, ctypes.POINTER(vp)]
        L.lfg_stretch_step_half.restype = ip
        L.lfg_stretch_step_half.argtypes = [vp, vp, ip, ip, f64, u64, u64, vp, vp, ctypes.POINTER(LfgTree), vp,
                                            vp, vp, sz, vp, ctypes.POINTER(vp)]
        L.lfg_stretch_step_half_spec.restype = ip
        L.lfg_stretch_step_half_spec.argtypes = [vp, vp, ip, ip, f64, u64, u64, vp, vp, ctypes.POINTER(LfgTree),
                                                 vp, vp, ip, ip, vp, sz, vp, ctypes.POINTER(vp)]
        L.lfg_stretch_step_shard.restype = ip
        L.lfg_stretch_step_shard.argtypes = [vp, ip, ip, f64, u64, u64, ip, ip, vp, vp, ctypes.POINTER(LfgTree),
                                             vp, vp, sz, vp, ctypes.POINTER(vp)]
        L.lfg_stretch_step_shard_spec.restype = ip
        L.lfg_stretch_step_shard_spec.argtypes = [vp, ip, ip, f64, u64, u64, ip, ip, vp, vp,
                                                  ctypes.POINTER(LfgTree), vp, ip, ip, vp, sz, vp, ctypes.POINTER(vp)]
        L.lfg_stretch_accept_regen_spec.restype = ip
        L.lfg_stretch_accept_regen_spec.argtypes = [vp, vp, ip, ip, f64, u64, u64, vp, vp, ctypes.POINTER(LfgTree),
                                                    ip, vp, sz, vp]
        L.lfg_stretch_step_shard_fold.restype = ip
        L.lfg_stretch_step_shard_fold.argtypes = [vp, vp, ip, ip, f64, u64, u64, ip, ip, vp, vp,
                                                  ctypes.POINTER(LfgTree), vp, vp, vp, vp, ip, ip, vp, sz, vp,
                                                  ctypes.POINTER(vp)]
        L.lfg_stretch_apply_verdicts.restype = ip
        L.lfg_stretch_apply_verdicts.argtypes = [vp, vp, ip, ip, ip, f64, u64, u64, vp, vp, vp]
        L.lfg_stretch_accept_regen.restype = ip
        L.lfg_stretch_accept_regen.argtypes = [vp, vp, ip, ip, ip, f64, u64, u64, vp, vp, vp]
        L.lfg_stretch_propose_dev.restype = ip
        L.lfg_stretch_propose_dev.argtypes = [vp, ip, ip, ip, f64, u64, vp, vp, vp, vp]
        L.lfg_stretch_accept_dev.restype = ip
        L.lfg_stretch_accept_dev.argtypes = [vp, vp, ip, ip, ip, vp, vp, vp, u64, vp, vp, vp]
        L.lfg_event_create.restype = ip
        L.lfg_event_create.argtypes = [ctypes.POINTER(vp)]
        L.lfg_event_destroy.restype = ip
        L.lfg_event_destroy.argtypes = [vp]
        L.lfg_event_elapsed_ms.restype = ip
        L.lfg_event_elapsed_ms.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_float)]
        L.lfg_wdphases.restype = ip
        L.lfg_wdphases.argtypes = [vp, vp, vp, ip, ip, vp, vp, vp, vp]
        L.lfg_gp_lnlike.restype = ip
        L.lfg_gp_lnlike.argtypes = [vp, vp, vp, ip, ip, vp, vp, ip, vp, vp]
        L.lfg_component_workspace_size.restype = sz
        L.lfg_component_workspace_size.argtypes = [ip, ip, ip, ip]
        L.lfg_component.restype = ip
        L.lfg_component.argtypes = [ip, vp, ip, vp, vp, ip, ip, ip, vp, vp, ip, vp, vp, vp, sz, vp]
        L.lfg_version.restype = ctypes.c_char_p
        L.lfg_version.argtypes = []
        L.lfg_layout.restype = ip
        L.lfg_layout.argtypes = [ctypes.POINTER(LfgTree)]
        if hasattr(L, "lfg_set_layout"):  # (older experiment builds lack it)
            L.lfg_set_layout.restype = ip
            L.lfg_set_layout.argtypes = [ip]
        _lib = L
        return L


def check(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed with code %d" % (what, rc))


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("lfit_python_amd needs a HIP GPU (MI355X): no device visible, "
                           "and the product path has no CPU fallback")


def stream_ptr(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Workspace:
    """Grow-only scratch buffer for the lfg_* entry points (one per device)."""

    _pool = {}

    @classmethod
    def get(cls, nbytes, device):
        import torch
        key = str(device)
        buf = cls._pool.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            cls._pool[key] = buf
        return buf
