"""Build / time compile-time variants of the fused passes (tuning aid, not product code).

  python tools/tune_variants.py build NAME=-DFLAG=1,-DOTHER=2 ...   # here: variants/libqsc_NAME.so
  python tools/tune_variants.py run [--config c3] [--names a,b]     # GPU box: one subprocess each

`run` times each variant's S-pass (fused Adam), C-pass and C-finish with HIP events on the
stream the kernels are launched on, checks that the solver state after a few iterations matches
the default build's (same NLLs), and prints one JSON line per variant.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "variants")
sys.path.insert(0, ROOT)


def cmd_build(specs):
    from quantized_spectrum_cartography_amd import _build
    os.makedirs(VDIR, exist_ok=True)
    for spec in specs:
        name, _, flags = spec.partition("=")
        fl = [f for f in flags.split(",") if f]
        _build.build(out=os.path.join(VDIR, "libqsc_%s.so" % name), extra_flags=fl, verbose=False)
        print("built", name, fl, flush=True)


def time_one(config, reps, tile=None):
    import torch
    from quantized_spectrum_cartography_amd import synthetic
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    I, J, K, R = synthetic.CONFIGS[config]
    prob = synthetic.onebit_problem(I, J, K, R, f=0.1, seed=20263, keep_T=False)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=R, tile=tile)
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=64)
    sol.run(10)
    torch.cuda.synchronize()
    st = sol.state()
    e = sol.engine

    def tk(fn):
        # launches captured in a hipGraph and replayed: device time, not Python launch time
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(reps):
                    fn()
            g.replay()
            s.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            g.replay()
            b.record(s)
            b.synchronize()
        torch.cuda.current_stream().wait_stream(s)
        return a.elapsed_time(b) / reps * 1e3

    us_s = tk(lambda: e.spass(sol.S, sol.C, 1, mS=sol.mS, vS=sol.vS, adam=sol.adam_s,
                              lambda_s=sol.lambda_s))
    us_c = tk(lambda: e.cpass(sol.S, sol.C))
    us_f = tk(lambda: e.cfinish(sol.C, 1, mC=sol.mC, vC=sol.vC, adam=sol.adam_c,
                                lambda_c=sol.lambda_c))
    us_sc = None
    if sol.fuse:
        us_sc = tk(lambda: e.scpass(sol.S, sol.C, sol.mS, sol.vS, sol.adam_s, sol.lambda_s))
    # end-to-end: 100 iterations as one prepared hipGraph replay (bench.py's timed region)
    sol.prepare(100)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    sol.run(100, use_graph=True)
    b.record()
    b.synchronize()
    gsps = 200 / (a.elapsed_time(b) * 1e-3)
    return dict(gsps=round(gsps), scfused_us=us_sc, spass_us=us_s, cpass_us=us_c,
                cfinish_us=us_f, nll_c=st["nll_c"],
                nll_s=st["nll_s"], nnz=obs.nnz, tile=obs.desc.PT,
                c_pad=round(obs.stats()["c_padding"], 3), s_pad=round(obs.stats()["s_padding"], 3))


def cmd_run(args):
    names = args.names.split(",") if args.names else sorted(
        f[len("libqsc_"):-3] for f in os.listdir(VDIR) if f.endswith(".so"))
    base = None
    for name in ["default"] + names:
        env = dict(os.environ)
        if name != "default":
            env["QSC_LIB_PATH"] = os.path.join(VDIR, "libqsc_%s.so" % name)
        cmd = [sys.executable, __file__, "_one", "--config", args.config, "--reps", str(args.reps)]
        if args.tile:
            cmd += ["--tile", str(args.tile)]
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(json.dumps({"variant": name, "rc": p.returncode, "err": p.stderr[-800:]}),
                  flush=True)
            if p.returncode < 0 or "illegal" in p.stderr or "fault" in p.stderr.lower():
                sys.exit(1)  # a GPU fault: start nothing more on the GPU
            continue
        r = json.loads(p.stdout.strip().splitlines()[-1])
        if base is None:
            base = r
        r["variant"] = name
        r["same_nll"] = (r["nll_c"] == base["nll_c"], r["nll_s"] == base["nll_s"])
        r["rel_nll"] = abs(r["nll_s"] - base["nll_s"]) / abs(base["nll_s"])
        print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run", "_one"])
    ap.add_argument("specs", nargs="*")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--names", default="")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--tile", type=int, default=0)
    args = ap.parse_args()
    if args.mode == "build":
        cmd_build(args.specs)
    elif args.mode == "run":
        cmd_run(args)
    else:
        print(json.dumps(time_one(args.config, args.reps, args.tile or None)))


if __name__ == "__main__":
    main()
