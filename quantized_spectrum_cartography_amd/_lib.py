"""ctypes binding of libqsc_hip.so (C ABI declared in include/qsc.h).

The argument types of every entry point are derived from the header itself, so the Python
binding and the C declaration cannot drift apart.  There is no CPU fallback: if the library
is missing or the device is not a gfx950, every product call raises.
"""
import ctypes
import os
import re
import threading

import torch  # noqa: F401  (must be imported first: torch's libamdhip64 is the process HIP runtime)

from . import _build

HEADER = os.path.join(os.path.dirname(_build.PKG_DIR), "include", "qsc.h")

QSC_MAX_BOUNDS = 256
QSC_MAX_R = 16
QSC_SLICE = 32  # S-format slice (pixel positions per list group), include/qsc.h
QSC_ENTRY_TAIL = 256  # pad entries after the last list (read-ahead tail), include/qsc.h
QSC_EINVAL = 100000
QSC_EUNSUPPORTED = 100001
LOSSES = {"probit": 0, "squared": 1}  # QSC_LOSS_PROBIT, QSC_LOSS_SQUARED
UNOBSERVED = 0xFF


class QscModel(ctypes.Structure):
    _fields_ = [("nbounds", ctypes.c_int32), ("log_model", ctypes.c_int32),
                ("sigma", ctypes.c_double), ("offset", ctypes.c_double),
                ("bounds", ctypes.c_float * QSC_MAX_BOUNDS), ("loss", ctypes.c_int32),
                ("reserved_", ctypes.c_int32)]


class QscAdam(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("project_nonneg", ctypes.c_int32),
                ("pad_", ctypes.c_int32)]


class QscObsDesc(ctypes.Structure):
    _fields_ = [("K", ctypes.c_int32), ("P", ctypes.c_int32), ("Pp", ctypes.c_int32),
                ("PT", ctypes.c_int32), ("ntiles", ctypes.c_int32), ("nks", ctypes.c_int32),
                ("wide", ctypes.c_int32), ("nbins", ctypes.c_int32), ("nnz", ctypes.c_int64),
                ("s_entries", ctypes.c_int64), ("c_entries", ctypes.c_int64),
                ("rowfmt", ctypes.c_int32), ("reserved_", ctypes.c_int32)]


# device-resident qsc_state: 4 int32 + 5 float + fused_fault int32 + fin_ticket uint64 + 4 reserved
STATE_BYTES = 64
STATE_FIELDS = ("step_c", "step_s", "iter", "pending", "normsq_s", "normsq_c", "nll_c", "nll_s",
                "normsq_s_prev")
STATE_OFFSETS = {name: 4 * i for i, name in enumerate(STATE_FIELDS)}

_HOST_STRUCTS = {"qsc_model": QscModel, "qsc_adam": QscAdam, "qsc_obs_desc": QscObsDesc}
_SCALARS = {"int": ctypes.c_int, "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64,
            "size_t": ctypes.c_size_t, "double": ctypes.c_double, "float": ctypes.c_float,
            "void": None}


def _ctype(decl):
    decl = decl.strip()
    decl = re.sub(r"\bconst\b", "", decl).strip()
    m = re.match(r"^([A-Za-z_][A-Za-z0-9_]*)\s*(\**)\s*[A-Za-z_0-9]*$", decl)
    if not m:
        raise ValueError("cannot parse C declaration %r" % decl)
    base, stars = m.group(1), m.group(2)
    if stars:
        if base in _HOST_STRUCTS:
            return ctypes.POINTER(_HOST_STRUCTS[base])
        if base == "char":
            return ctypes.c_char_p
        return ctypes.c_void_p  # device pointers, streams, workspaces
    return _SCALARS[base]


def parse_header(path=HEADER):
    """Return {name: (restype, [argtypes])} for every QSC_API function in the header."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"QSC_API\s+([^;(]*?)\b(qsc_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src, re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        args = " ".join(args.split())
        argtypes = [] if args in ("", "void") else [_ctype(a) for a in args.split(",")]
        out[name] = (_ctype(ret + " x"), argtypes)
    return out


class QscError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def lib():
    """Load libqsc_hip.so (building it first if it is missing and hipcc is available)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("QSC_LIB_PATH", _build.LIB_PATH)  # variant builds (tuning)
        if not os.path.exists(path):
            try:
                _build.build(verbose=False)
            except Exception as e:  # pragma: no cover - depends on toolchain
                raise QscError("libqsc_hip.so is missing and could not be built: %s" % e)
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        missing = []
        for name, (res, args) in parse_header().items():
            fn = getattr(L, name, None)
            if fn is None:  # an older variant library (QSC_LIB_PATH): fails when called
                missing.append(name)
                continue
            fn.restype = res
            fn.argtypes = args
        L.qsc_missing_ = missing
        _lib = L
    return _lib


def err(code):
    s = lib().qsc_error_string(int(code))
    return s.decode() if s else "error %d" % code


# QSC_DEBUG_CHECK=1 (with a QSC_DEBUG=1 library, _build.py --debug): after every call outside
# graph capture, synchronise and raise if a kernel bounds check failed (qsc_debug_status)
_DEBUG_CHECK = os.environ.get("QSC_DEBUG_CHECK", "0") == "1"


def call(name, *args):
    """Call a qsc_* entry point and raise QscError on a non-zero status."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise QscError("%s failed: %s (code %d)" % (name, err(rc), rc))
    if _DEBUG_CHECK and not torch.cuda.is_current_stream_capturing():
        line = lib().qsc_debug_status(1)
        if line > 0:
            raise QscError("%s: kernel bounds check failed at qsc_pass.hip:%d (QSC_DEBUG)"
                           % (name, line))
    return rc


_checked_devices = set()


def require_device(t):
    """Fail loudly unless tensor t lives on a gfx950 GPU the library can run on."""
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise QscError("the HIP hot path needs GPU tensors (got %s)" %
                       (t.device if isinstance(t, torch.Tensor) else type(t)))
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    if dev not in _checked_devices:
        call("qsc_device_check", dev)
        _checked_devices.add(dev)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def make_model(bin_boundaries, noise_std, offset=0.0, log_model=False, loss="probit"):
    b = bin_boundaries
    if isinstance(b, torch.Tensor):
        b = b.detach().to("cpu", torch.float32).tolist()
    b = [float(x) for x in b]
    if not 2 <= len(b) <= QSC_MAX_BOUNDS:
        raise ValueError("need 2..%d bin boundaries, got %d" % (QSC_MAX_BOUNDS, len(b)))
    m = QscModel()
    m.nbounds = len(b)
    m.log_model = 1 if log_model else 0
    m.sigma = float(noise_std)
    m.offset = float(offset or 0.0)
    if loss not in LOSSES:
        raise ValueError("loss must be one of %s" % sorted(LOSSES))
    m.loss = LOSSES[loss]
    for i, x in enumerate(b):
        m.bounds[i] = x
    return m


def make_adam(lr, betas=(0.9, 0.999), eps=1e-8, project_nonneg=False):
    a = QscAdam()
    a.lr, a.beta1, a.beta2, a.eps = float(lr), float(betas[0]), float(betas[1]), float(eps)
    a.project_nonneg = 1 if project_nonneg else 0
    return a


def read_state(st):
    """Decode a device qsc_state tensor (uint8[64]) into a dict (synchronises)."""
    raw = st.detach().cpu()
    ints = raw[:16].view(torch.int32).tolist()
    flts = raw[16:36].view(torch.float32).tolist()
    out = dict(zip(STATE_FIELDS, ints + flts))
    out["fused_fault"] = int(raw[36:40].view(torch.int32).item())
    return out


def state_field(st, name):
    """A 1-element device view of one float field of a qsc_state tensor."""
    o = STATE_OFFSETS[name]
    return st[o:o + 4].view(torch.float32)
