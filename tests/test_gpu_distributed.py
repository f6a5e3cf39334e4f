"""GPU: the sharded solvers on a real RCCL process group (world size 1 on the one-GPU test box;
the N > 1 logic itself is covered by tests/test_distributed_gloo.py).

With one rank the collectives are identities, so each sharded solver must reproduce the
single-GPU FreeSSolver: IJ-slab bit for bit (same kernels, the C update through qsc_cupdate),
K-slab to the parity tolerance (its S update runs from the materialised gradient).  The runs
also exercise hipGraph capture of the iteration including the RCCL all-reduce.
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import rel_fro

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def _problem():
    from quantized_spectrum_cartography_amd import synthetic
    return synthetic.onebit_problem(64, 48, 96, 5, f=0.2, seed=77)


def _reference(prob, iters):
    from quantized_spectrum_cartography_amd.obs import Observations
    from quantized_spectrum_cartography_amd.qmc import FreeSSolver
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=5)
    sol = FreeSSolver(obs, prob["S0"], prob["C0"], hist_cap=iters + 2)
    sol.run(iters)
    return sol.S_pixels().cpu().numpy(), sol.C.cpu().numpy(), sol.history()


@pytest.mark.parametrize("use_graph", [False, True])
def test_ijslab_world1_equals_single_gpu(pg, use_graph):
    from quantized_spectrum_cartography_amd.distributed import IJSlabSolver
    from quantized_spectrum_cartography_amd.obs import Observations
    prob = _problem()
    iters = 10
    S_ref, C_ref, (cc_ref, cs_ref) = _reference(prob, iters)
    obs = Observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], R_hint=5)
    sol = IJSlabSolver(obs, prob["S0"], prob["C0"], dist=pg, hist_cap=iters + 2)
    sol.run(iters, use_graph=use_graph)
    torch.cuda.synchronize()
    assert np.array_equal(sol.S_pixels().cpu().numpy(), S_ref)
    assert np.array_equal(sol.C.cpu().numpy(), C_ref)
    cc, cs = sol.history()
    assert np.allclose(cc, cc_ref, rtol=1e-6) and np.allclose(cs, cs_ref, rtol=1e-6)
    if use_graph:
        # the whole run (fused S-step + C-pass launches + RCCL) as one captured hipGraph
        assert sol._graphs.get(iters) is not None, sol.graph_error


def test_kslab_world1_matches_single_gpu(pg):
    from quantized_spectrum_cartography_amd.distributed import KSlabSolver, kslab_observations
    prob = _problem()
    iters = 10
    S_ref, C_ref, _ = _reference(prob, iters)
    obs = kslab_observations(prob["Y"], prob["Wx"], prob["b"], prob["sigma"], pg, R_hint=5)
    sol = KSlabSolver(obs, prob["S0"], prob["C0"], dist=pg, hist_cap=iters + 2)
    sol.run(iters, use_graph=True)
    torch.cuda.synchronize()
    assert rel_fro(sol.S_pixels().cpu().numpy(), S_ref) < 1e-5
    assert rel_fro(sol.C.cpu().numpy(), C_ref) < 1e-5
