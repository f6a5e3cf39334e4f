"""Build variant libraries in parallel (diagnostic / A-B runs):
  python tools/build_variants.py name:-DFLAG=1,-DOTHER=2 name2:-DX=1
Each lands in variants/libqsc_<name>.so (loaded through QSC_LIB_PATH)."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantized_spectrum_cartography_amd import _build  # noqa: E402


def one(spec):
    name, _, flags = spec.partition(":")
    out = os.path.join("variants", "libqsc_%s.so" % name)
    _build.build(out=out, extra_flags=[f for f in flags.split(",") if f], verbose=False)
    return out


if __name__ == "__main__":
    os.makedirs("variants", exist_ok=True)
    with ThreadPoolExecutor(max_workers=3) as ex:
        for out in ex.map(one, sys.argv[1:]):
            print(out, flush=True)
