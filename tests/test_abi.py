"""CPU: the C-ABI library builds for gfx950, loads, and exports every symbol of include/qsc.h;
ctypes struct layouts agree with the C compiler's.  No compute calls (no GPU here)."""
import ctypes
import os
import subprocess
import tempfile

import pytest

from quantized_spectrum_cartography_amd import _build, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def libpath():
    return _build.build(verbose=False)


def test_header_parses_all_entry_points():
    h = _lib.parse_header()
    for name in ("qsc_spass", "qsc_cpass", "qsc_cfinish", "qsc_quantize",
                 "qsc_prob_probit", "qsc_reconstruct", "qsc_gram", "qsc_chol_solve",
                 "qsc_obs_layout", "qsc_supdate", "qsc_state_flush"):
        assert name in h
    assert len(h) >= 30


def test_library_exports_every_declared_symbol(libpath):
    out = subprocess.check_output(["nm", "-D", "--defined-only", libpath]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = sorted(set(_lib.parse_header()) - exported)
    assert not missing, missing


def test_library_loads_and_reports(libpath):
    L = _lib.lib()
    assert L.qsc_version() >= 1
    assert L.qsc_error_string(0) == b"success"
    assert L.qsc_error_string(_lib.QSC_EINVAL) == b"invalid argument"


def test_code_object_targets_gfx950(libpath):
    # the fat binary carries a gfx950 code object (bundle id amdgcn-amd-amdhsa--gfx950)
    data = open(libpath, "rb").read()
    assert b"gfx950" in data


def test_struct_layouts_match_c():
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "qsc.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(qsc_model), sizeof(qsc_adam),
         sizeof(qsc_obs_desc), sizeof(qsc_state), offsetof(qsc_model, bounds),
         offsetof(qsc_obs_desc, nnz), offsetof(qsc_state, fused_fault),
         offsetof(qsc_state, fin_ticket));
  return 0;
}
'''
    d = tempfile.mkdtemp()
    c = os.path.join(d, "t.c")
    exe = os.path.join(d, "t")
    open(c, "w").write(src)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
    vals = [int(x) for x in subprocess.check_output([exe]).split()]
    assert vals[0] == ctypes.sizeof(_lib.QscModel)
    assert vals[1] == ctypes.sizeof(_lib.QscAdam)
    assert vals[2] == ctypes.sizeof(_lib.QscObsDesc)
    assert vals[3] == _lib.STATE_BYTES
    assert vals[4] == _lib.QscModel.bounds.offset
    assert vals[5] == _lib.QscObsDesc.nnz.offset
    # the words _lib.read_state decodes by index (the persistent loop's fault word: int word 9;
    # the reserved 64-bit word 5)
    assert vals[6] == 36 and vals[7] == 40


def test_product_fails_loudly_without_gpu():
    import torch
    from quantized_spectrum_cartography_amd import quantization_model as qm
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.QscError):
        qm.get_tensor(torch.rand(2, 1, 4, 4), torch.rand(2, 3))


def test_host_constants_match_header():
    """Host-side buffer sizing uses these constants (e.g. s_width has Pp / QSC_SLICE entries):
    they must equal the header's #defines."""
    import re
    src = open(_lib.HEADER).read()
    defs = dict(re.findall(r"#define\s+(QSC_[A-Z0-9_]+)\s+(0x[0-9A-Fa-f]+|\d+)\b", src))
    assert int(defs["QSC_SLICE"]) == _lib.QSC_SLICE
    assert int(defs["QSC_ENTRY_TAIL"]) == _lib.QSC_ENTRY_TAIL
    assert int(defs["QSC_MAX_R"]) == _lib.QSC_MAX_R
    assert int(defs["QSC_MAX_BOUNDS"]) == _lib.QSC_MAX_BOUNDS
    assert int(defs["QSC_EINVAL"]) == _lib.QSC_EINVAL
    assert int(defs["QSC_UNOBSERVED"], 0) == _lib.UNOBSERVED


def _c_sizeof_model():
    src = '#include <stdio.h>\n#include "qsc.h"\nint main(void){printf("%zu %zu\\n", ' \
          'sizeof(qsc_model), offsetof(qsc_model, loss));return 0;}\n'
    d = tempfile.mkdtemp()
    c, exe = os.path.join(d, "m.c"), os.path.join(d, "m")
    open(c, "w").write("#include <stddef.h>\n" + src)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
    return [int(x) for x in subprocess.check_output([exe]).split()]


def test_integration_stub_struct_matches_c():
    """The reference-side ctypes stub documented in INTEGRATION.md section 3 declares the same
    qsc_model as the C header: exec the snippet's struct definition and compare sizes."""
    import re
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    struct_src = re.search(r"(class _Model\(ctypes\.Structure\):.*?\]\n)", text, re.S).group(1)
    ns = {"ctypes": ctypes}
    exec(struct_src, ns)
    size, loss_off = _c_sizeof_model()
    assert ctypes.sizeof(ns["_Model"]) == size
    assert ns["_Model"].loss.offset == loss_off


def test_integration_stub_error_path(libpath):
    """The stub's error path turns a return code into its message:
    exec the snippet's qsc_error_string declarations against the built library."""
    import re
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    decl = "\n".join(re.findall(r"^_L\.qsc_error_string\..*$", text, re.M))
    assert "restype = ctypes.c_char_p" in decl
    ns = {"ctypes": ctypes, "_L": ctypes.CDLL(libpath)}
    exec(decl, ns)
    assert ns["_L"].qsc_error_string(_lib.QSC_EINVAL).decode() == "invalid argument"


def _param_list(sig):
    """The top-level parameter list of a demangled function signature."""
    depth, end = 0, None
    for i in range(len(sig) - 1, -1, -1):
        c = sig[i]
        if c == ")":
            if depth == 0:
                end = i
            depth += 1
        elif c == "(":
            depth -= 1
            if depth == 0:
                return sig[i + 1:end]
    return ""


def test_kernels_take_no_reference_parameters(libpath):
    """A __global__ function's reference parameter is passed as a host address that the device
    then dereferences (a memory-access fault).  Every kernel of the library takes its structs by
    value: scan the code object's kernel symbols (ours live in an anonymous namespace)."""
    import re
    data = open(libpath, "rb").read()
    names = sorted(set(re.findall(rb"_ZN12_GLOBAL__N_1[0-9A-Za-z_]*_kernel[0-9A-Za-z_]*", data)))
    assert len(names) > 20
    out = subprocess.run(["c++filt"], input=b"\n".join(names), capture_output=True,
                         check=True).stdout.decode().split("\n")
    bad = [s for s in out if s and "&" in _param_list(s)]
    assert not bad, bad[:3]
