"""Build libqsc_hip.so (the gfx950 HIP kernels + C ABI) in-tree with hipcc.

The shared library lands next to this file so that it travels with the repository snapshot
to the GPU box (it is git-ignored, not gpurun-ignored).  No torch extension machinery is
involved: the boundary is a plain C ABI (include/qsc.h) bound with ctypes.
"""
import os
import shutil
import subprocess
import sys
import tempfile

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libqsc_hip.so")
SOURCES = ["qsc_ops.hip", "qsc_obs.hip", "qsc_pass.hip", "qsc_gram.hip", "qsc_spa.hip",
           "qsc_map.hip"]
ARCH = os.environ.get("QSC_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: hipcc contracts a*b+c into FMA by default, which would change the
# reference's separately rounded products and sums (get_tensor, quantize); FMAs that are
# wanted are written explicitly with __builtin_fmaf.  -fno-slp-vectorize: pairing scalar f32
# lanes into v_pk_* ops costs a v_mov per operand and s_nop hazards in the fused passes.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall",
          "-Wno-unused-function", "-ffp-contract=off", "-fno-slp-vectorize"]
# per-source flags.  qsc_pass.hip (the fused passes) runs with f32 denormals flushed: the
# one-bit likelihood carries its tail probability 2^-101 low so that tails below 2^-25 (where the
# reference's fp32 erf saturates, P == 0) underflow to exactly 0 without a compare per entry
# (QSC_FTZ_SAT, qsc_common.cuh lik_grad2).
FILE_FLAGS = {"qsc_pass.hip": ["-fgpu-flush-denormals-to-zero", "-DQSC_FTZ_SAT=1"]}


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP kernels of quantized_spectrum_cartography_amd "
                       "need ROCm's hipcc to build")


def _stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(os.path.dirname(PKG_DIR), "include", "qsc.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=True, out=None, extra_flags=(), link_flags=()):
    """Compile every HIP source for gfx950 and link libqsc_hip.so (parallel, one hipcc per file).

    `out` / `extra_flags` produce a variant library (e.g. -DQSC_SPASS_WAVES=4 for tuning runs,
    loaded through QSC_LIB_PATH); the default build is always the in-tree LIB_PATH."""
    lib_path = out or LIB_PATH
    if out is None and not force and not _stale():
        return LIB_PATH
    hipcc = _hipcc()
    tmp = tempfile.mkdtemp(prefix="qsc_build_")
    try:
        procs = []
        objs = []
        for src in SOURCES:
            obj = os.path.join(tmp, src.replace(".hip", ".o"))
            objs.append(obj)
            cmd = ([hipcc] + CFLAGS + FILE_FLAGS.get(src, []) + list(extra_flags) +
                   ["-c", os.path.join(CSRC, src), "-o", obj])
            procs.append((src, cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                                     stderr=subprocess.STDOUT)))
        failed = []
        for src, cmd, p in procs:
            out, _ = p.communicate()
            if p.returncode != 0:
                failed.append((src, out.decode(errors="replace")))
            elif verbose and out:
                sys.stderr.write(out.decode(errors="replace"))
        if failed:
            msg = "\n".join("---- %s ----\n%s" % f for f in failed)
            raise RuntimeError("hipcc failed:\n" + msg)
        out_tmp = lib_path + ".tmp"
        cmd = ([hipcc, "-shared", "-fPIC", "--offload-arch=" + ARCH] + list(link_flags) + objs +
               ["-o", out_tmp])
        subprocess.check_call(cmd)
        os.replace(out_tmp, lib_path)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if verbose:
        print("built", lib_path)
    return lib_path


# Debug variants: QSC_DEBUG=1 bounds checks in the pass kernels
# (qsc_common.cuh QSC_DCHECK, read back with qsc_debug_status); "asan" adds AddressSanitizer to
# the HOST code of the C ABI (argument checks, workspace carving, the host scheduler), loaded
# with the clang ASan runtime preloaded (tools/asan_check.sh).  Device code is never sanitized.
DEBUG_FLAGS = ["-DQSC_DEBUG=1", "-g"]
ASAN_FLAGS = DEBUG_FLAGS + ["-Xarch_host", "-fsanitize=address", "-fno-omit-frame-pointer"]
DEBUG_LIB = os.path.join(PKG_DIR, "libqsc_hip_debug.so")
ASAN_LIB = os.path.join(PKG_DIR, "libqsc_hip_asan.so")


def build_variant(kind):
    """kind "debug" -> libqsc_hip_debug.so, "asan" -> libqsc_hip_asan.so (next to the release
    library; select one with QSC_LIB_PATH)."""
    if kind == "debug":
        return build(out=DEBUG_LIB, extra_flags=DEBUG_FLAGS, verbose=False)
    if kind == "asan":
        return build(out=ASAN_LIB, extra_flags=ASAN_FLAGS, verbose=False,
                     link_flags=["-Xarch_host", "-fsanitize=address", "-shared-libsan"])
    raise ValueError(kind)


if __name__ == "__main__":
    if "--debug" in sys.argv:
        print("built", build_variant("debug"))
    elif "--asan" in sys.argv:
        print("built", build_variant("asan"))
    else:
        build(force="--force" in sys.argv)
