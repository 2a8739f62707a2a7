"""Round-2 diagnostics on the GPU box: persistent-engine barrier timestamps on C2 / C4."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from simgrid_amd import lmm as L  # noqa: E402
from simgrid_amd import multi as M  # noqa: E402

what = sys.argv[1]
if what not in ("c2", "c4"):
    sys.exit("usage: diag_r2.py c2|c4  (the C5 shard diagnostics moved to tests/test_gpu_multi.py)")
if True:
    s = L.System(False)
    if what == "c2":
        s.gen_synthetic(1_000_000, 10_000_000, 8, seed=1, want_vars=False)
    else:
        s.gen_platform_flows(L.platform_params(topology=L.FAT_TREE, topo_parameters="3;16,16,16;1,16,16;1,1,1",
                                               loopback_bw=1e8, model=L.LV08, n_flows=100_000, seed=1),
                             want_vars=False)
    s.prepare()
    s.device_solve()
    s.persist_profile(True)
    for _ in range(3):
        s.device_solve()
    t = s.persist_profile(False)
    np.save(f"gpurun_out/persist_blocks_{what}.npy", s.persist_profile_blocks())
    st = s.last_stats()
    arr, ext = t[:, 0].astype(np.float64), t[:, 1].astype(np.float64)
    # barrier g >= 1: phase time = last arrival(g) - exit(g-1); barrier time = exit(g) - last arrival(g)
    ph = (arr[1:] - ext[:-1]) / 100.0  # us
    br = (ext[1:] - arr[1:]) / 100.0
    out = dict(workload=what, device_ms=st["device_ms"], rounds=st["rounds"], barriers=len(t) - 1,
               total_us=float((ext[-1] - ext[0]) / 100.0), phase_us=ph.tolist(), barrier_us=br.tolist())
    with open(f"gpurun_out/persist_{what}.json", "w") as fo:
        json.dump(out, fo)
    print(what, st, "sum phase", ph.sum(), "sum barrier", br.sum(), flush=True)
