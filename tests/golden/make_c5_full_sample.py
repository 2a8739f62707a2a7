"""Generate tests/golden/c5_full_sample.npz: the oracle's solution of the full-size C5 system.

C5 (BASELINE.json configs[4]): FairBottleneck (fair_bottleneck.cpp:23-153) over 1e7 L07 flows on the dragonfly
8,4;16,3;8,2;4 (tests/test_gpu_configs.py C5_PLATFORM, seed 1).  The oracle builds the system with its own
restatement of the platform and flow model (oracle/platforms.py) and solves it once on the CPU
(oracle/lmm_oracle.cpp's bottleneck_solve restatement: a few minutes).  The fixture keeps:

  * `sample_idx` / `sample_x`: 100,000 flow indices (generation order, fixed RNG) and their oracle values — the
    one-context device solve is bit-identical to the reference's element order, so the GPU test requires these
    bytes exactly;
  * `flat_sha256`: sha256 of the product's flattened system for the same parameters (var_ptr, cnst_idx,
    weight, penalty, vbound, cbound, cflags and the reference-order CSC permutation), so the GPU test knows it
    solved the very same system;
  * `oracle_rounds`, `oracle_seconds`: the oracle's round count and solve time (this container's CPU).

Run from the repo root (CPU only, ~20 GB of host memory at peak):  python tests/golden/make_c5_full_sample.py
"""
import hashlib
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

NFLOWS, SEED = 10_000_000, 1
NSAMPLE = 100_000
SAMPLE_SEED = 20261018
OUT = os.path.join(ROOT, "tests", "golden", "c5_full_sample.npz")
C5_TOPO = "8,4;16,3;8,2;4"


def flat_sha256(f):
    h = hashlib.sha256()
    for a in (f.var_ptr, f.cnst_idx, f.weight, f.penalty, f.vbound, f.cbound, f.cflags, f.csc_order):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def params(mod):
    return mod.platform_params(topology=mod.DRAGONFLY, topo_parameters=C5_TOPO, loopback_bw=1e9, limiter_bw=2e8,
                               model=mod.L07, n_flows=NFLOWS, seed=SEED)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    import __graft_entry__

    __graft_entry__.build()
    from oracle import pyoracle as O
    from simgrid_amd import lmm as L
    from simgrid_amd import multi as M

    L.set_precision(1e-5)
    O.set_precision(1e-5)
    t0 = time.time()
    ps = L.System(False, L.System.FAIR_BOTTLENECK)
    _, pv = ps.gen_platform_flows(params(L))
    f = M.export_flat(ps)
    assert len(f.penalty) == NFLOWS and np.array_equal(f.var_ids, pv), "flat order must be generation order"
    sha = flat_sha256(f)
    print(f"product system built + exported in {time.time() - t0:.1f} s, nnz {len(f.weight)}, sha {sha[:16]}",
          flush=True)
    del ps, f

    os_ = O.System(False, O.System.FAIR_BOTTLENECK)
    t1 = time.time()
    _, vs = os_.gen_platform_flows(params(O))
    print(f"oracle system built in {time.time() - t1:.1f} s", flush=True)
    secs = os_.timed_solve()
    rounds = os_.last_rounds
    print(f"oracle solve {secs:.1f} s, {rounds} rounds", flush=True)
    y = os_.values_of(vs, NFLOWS)
    del os_
    rng = np.random.default_rng(SAMPLE_SEED)
    idx = np.sort(rng.choice(NFLOWS, NSAMPLE, replace=False)).astype(np.int64)
    np.savez_compressed(OUT, sample_idx=idx, sample_x=y[idx], flat_sha256=np.array(sha),
                        oracle_rounds=np.int64(rounds), oracle_seconds=np.float64(secs),
                        oracle_cpu=np.array(cpu_model()), n_flows=np.int64(NFLOWS),
                        all_positive=np.bool_(bool(np.all(y > 0))), x_sum=np.float64(np.sum(y)))
    print(f"wrote {OUT}: {NSAMPLE} samples, x in [{y.min():.6g}, {y.max():.6g}]", flush=True)


if __name__ == "__main__":
    main()
