#!/bin/bash
# Round 6: the round kernels' state stores written through (build knob LMM_WT=1, abl/wt) against the product build —
# does the launch boundary's release get cheaper with fewer dirty L2 lines?  Engine bit-identity and C2 parity with the
# WT build first, then same-box A/B on C2 / C2 stress, then the C2 anatomy of both (boundary gaps).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 200 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
LMM_AMD_LIB=abl/wt/liblmm_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_engines.py tests/test_gpu_parity.py \
  -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06_tests_m.log 2>&1 \
  || { tail -30 gpurun_out/r06_tests_m.log; exit 1; }
tail -n 2 gpurun_out/r06_tests_m.log
C2="--steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0"
for pass in 1 2; do
  step abm_c2_base_$pass 200 python bench.py $C2
  step abm_c2_wt_$pass 200 env LMM_AMD_LIB=abl/wt/liblmm_amd.so python bench.py $C2
done
step abm_c2s_base 200 python bench.py --variant stress $C2
step abm_c2s_wt 200 env LMM_AMD_LIB=abl/wt/liblmm_amd.so python bench.py --variant stress $C2
step abm_c4_base_1 200 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
step abm_c4_wt_1 200 env LMM_AMD_LIB=abl/wt/liblmm_amd.so python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
step prof_c2m 200 env LMM_AMD_LIB=abl/wt/liblmm_amd.so python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/r06_prof_c2m.json
step anat_c2m_wt 200 env LMMHIP_SAT_BLOCKS=1024 LMM_AMD_LIB=abl/wtanat/liblmm_amd.so python scripts/anatomy.py \
  --rounds 70,71,200,201 --product-profile gpurun_out/r06_prof_c2m.json --out gpurun_out/r06_c2_round_anatomy_m_wt.json \
  --raw gpurun_out/r06_anat_c2m_wt.npz
step anat_c2m_base 200 env LMMHIP_SAT_BLOCKS=1024 LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py \
  --rounds 70,71,200,201 --out gpurun_out/r06_c2_round_anatomy_m_base.json --raw gpurun_out/r06_anat_c2m_base.npz
