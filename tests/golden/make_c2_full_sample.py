"""Generate tests/golden/c2_full_sample.npz: the oracle's solution of the full-size C2 system.

C2 (BASELINE.json configs[1]): the synthetic maxmin_bench-style system, 1e6 constraints x 1e7 variables x 8
elements, seed 1, plain variant (lmm_generators.hpp `synthetic`).  The oracle (oracle/lmm_oracle.cpp, the
statement-level restatement of maxmin.cpp:487-693) solves it once on the CPU (~10-15 minutes: the reference's
light-table rescan is O(rounds x constraints), maxmin.cpp:663-680).  The fixture keeps:

  * `sample_idx` / `sample_x`: 100,000 variable indices (generation order, fixed RNG) and their oracle values;
  * `sat_bits`: the saturated-constraint bitmap of the oracle solution (np.packbits over constraint ids, the
    flattened constraint order = creation order for this generator), computed with the reference's test
    `bound - usage <= bound * prec` (maxmin.cpp print()) over the flattened system;
  * `csr_sha256`: sha256 of the flattened system's structure and numbers (var_ptr, cnst_idx, weight,
    penalty, vbound, cbound, cflags), so the GPU test knows it solved the very same system;
  * `oracle_rounds`, `oracle_seconds`: the oracle's sequential round count and solve time.

Run from the repo root (CPU only, ~30 GB of host memory at peak):  python tests/golden/make_c2_full_sample.py
(--stress: the stress variant, tests/golden/c2_stress_full_sample.npz)

Round 4 changed the flattened system's constraint rule (System::flatten_maxmin: every listed constraint a
member lies on is flattened, whatever its bound; the ~1000 zero-bound constraints of C2 start dead in the
solver's init instead of being left out).  The oracle solution does not depend on the flatten, so the fixture
was converted rather than re-solved (`--convert-superset`): the new flat, filtered back to the constraints that
pass the part test, must hash to the stored `csr_sha256` of the old rule; the zero-bound constraints are
saturated by the reference's test (0 - usage > 0 never holds) and the other bits keep their order.
"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

NC, NV, K, SEED = 1_000_000, 10_000_000, 8, 1
NSAMPLE = 100_000
SAMPLE_SEED = 20261017
OUT = os.path.join(ROOT, "tests", "golden", "c2_full_sample.npz")
# --stress: the C2 stress variant (bench.py --variant stress: 5 % FATPIPE constraints, 10 % bounded variables,
# penalties {1, 2, 4}) into c2_stress_full_sample.npz (round 5)
STRESS_KW = dict(penalty_mix=1, bounded_permille=100, fatpipe_permille=50)
GEN_KW = {}
if "--stress" in sys.argv:
    GEN_KW = STRESS_KW
    OUT = os.path.join(ROOT, "tests", "golden", "c2_stress_full_sample.npz")


def flat_sha256(f):
    h = hashlib.sha256()
    for a in (f.var_ptr, f.cnst_idx, f.weight, f.penalty, f.vbound, f.cbound, f.cflags):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def saturated_bits(f, x, prec):
    """Saturated constraints of the flat system `f` under dense values `x` (tests/test_gpu_parity.py's
    saturated_dense, as a bitmap over constraint ids)."""
    rows = np.repeat(np.arange(len(f.penalty)), np.diff(f.var_ptr))
    wx = f.weight * x[rows]
    use = np.bincount(f.cnst_idx, weights=wx, minlength=len(f.cbound))
    fat = (f.cflags & 1).astype(bool)
    if fat.any():
        mx = np.zeros(len(f.cbound))
        np.maximum.at(mx, f.cnst_idx, wx)
        use = np.where(fat, mx, use)
    sat = ~(f.cbound - use > f.cbound * prec)
    return np.packbits(sat.astype(np.uint8))


def part_only(f, prec):
    """`f` without the constraints that fail the part test (the pre-round-4 flatten rule)."""
    from simgrid_amd import multi as M

    keep = f.cbound > f.cbound * prec
    newid = np.cumsum(keep) - 1
    ek = keep[f.cnst_idx]
    rows = np.repeat(np.arange(len(f.penalty)), np.diff(f.var_ptr))
    var_ptr = np.zeros(len(f.penalty) + 1, np.int64)
    np.cumsum(np.bincount(rows[ek], minlength=len(f.penalty)), out=var_ptr[1:])
    return M.Flat(var_ptr, newid[f.cnst_idx[ek]].astype(np.int32), f.weight[ek], f.penalty, f.vbound,
                  f.cbound[keep], f.cflags[keep], f.var_ids), keep


def convert_superset():
    import __graft_entry__

    __graft_entry__.build()
    from simgrid_amd import lmm as L
    from simgrid_amd import multi as M

    L.set_precision(1e-5)
    fx = dict(np.load(OUT))
    ps = L.System(False)
    ps.gen_synthetic(NC, NV, K, seed=SEED)
    f = M.export_flat(ps)
    del ps
    old, keep = part_only(f, 1e-5)
    assert flat_sha256(old) == str(fx["csr_sha256"]), "the part-only filter does not give the solved system"
    old_bits = np.unpackbits(fx["sat_bits"])[: int(keep.sum())].astype(bool)
    sat = np.ones(len(f.cbound), bool)
    sat[keep] = old_bits
    fx["sat_bits"] = np.packbits(sat.astype(np.uint8))
    fx["csr_sha256"] = np.array(flat_sha256(f))
    fx["n_saturated"] = np.int64(sat.sum())
    np.savez_compressed(OUT, **fx)
    print(f"converted {OUT}: {len(f.cbound)} constraints ({int((~keep).sum())} zero-bound), "
          f"{int(sat.sum())} saturated", flush=True)


def main():
    import __graft_entry__

    __graft_entry__.build()
    from oracle import pyoracle as O
    from simgrid_amd import lmm as L
    from simgrid_amd import multi as M

    L.set_precision(1e-5)
    O.set_precision(1e-5)
    t0 = time.time()
    ps = L.System(False)
    pv = ps.gen_synthetic(NC, NV, K, seed=SEED, **GEN_KW)
    f = M.export_flat(ps)
    assert len(f.penalty) == NV and np.array_equal(f.var_ids, pv), "flat order must be generation order"
    sha = flat_sha256(f)
    print(f"product system built + exported in {time.time() - t0:.1f} s, sha {sha[:16]}", flush=True)
    del ps

    os_ = O.System(False)
    vs = os_.gen_synthetic(NC, NV, K, seed=SEED, **GEN_KW)
    t1 = time.time()
    secs = os_.timed_solve()
    rounds = os_.last_rounds
    print(f"oracle solve {secs:.1f} s ({time.time() - t1:.1f} s wall), {rounds} rounds", flush=True)
    y = os_.values_of(vs, NV)
    del os_
    rng = np.random.default_rng(SAMPLE_SEED)
    idx = np.sort(rng.choice(NV, NSAMPLE, replace=False)).astype(np.int64)
    bits = saturated_bits(f, y, 1e-5)
    np.savez_compressed(OUT, sample_idx=idx, sample_x=y[idx], sat_bits=bits, csr_sha256=np.array(sha),
                        oracle_rounds=np.int64(rounds), oracle_seconds=np.float64(secs),
                        n_saturated=np.int64(np.unpackbits(bits)[:NC].sum()))
    print(f"wrote {OUT}: {NSAMPLE} samples, {int(np.unpackbits(bits)[:NC].sum())} saturated constraints",
          flush=True)


if __name__ == "__main__":
    if "--convert-superset" in sys.argv:
        convert_superset()
    else:
        main()
