#!/bin/bash
# Round 6, second GPU pass: same-box A/B of the tail levers the round anatomy named (abl/base: round-5 vote queue +
# saturation loop; abl/rdq: + the vote's wave-aggregated ready queue; abl/pipe: + the saturation's pipelined
# candidate loads; the product build: + the update's candidates in 8 lists instead of ~1,024 segments), C2 and C2
# stress; the C2 anatomy of the new build (raw records too), the C4 anatomy
# (frontier engine), and the dependency-depth comparison (oracle depth vs device rounds, scripts/depth.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.log"
  local rc=$?
  tail -c 300 "gpurun_out/$name.out"; echo
  if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
for pass in 1 2; do
  for v in base rdq pipe new; do
    lib=abl/$v/liblmm_amd.so; [ $v = new ] && lib=simgrid_amd/_lib/liblmm_amd.so
    step ab_c2_${v}_$pass 200 env LMM_AMD_LIB=$lib python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
  done
done
for v in base new; do
  lib=abl/$v/liblmm_amd.so; [ $v = new ] && lib=simgrid_amd/_lib/liblmm_amd.so
  step ab_c2s_$v 200 env LMM_AMD_LIB=$lib python bench.py --variant stress --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
done
# knobs on the new build: the stamps' vote below 5e5 alive rows; 6 saturation workgroups per CU
step ab_c2_vbr 200 env LMMHIP_VOTE_BITS_ROWS=500000 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
step ab_c2_sb6 200 env LMMHIP_SAT_BLOCKS=1536 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0
step prof_c2b 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dropin-steps 0 --profile-json gpurun_out/r06_prof_c2b.json
step anat_c2b 200 env LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --rounds 70,71,200,201 \
  --product-profile gpurun_out/r06_prof_c2b.json --out gpurun_out/r06_c2_round_anatomy_b.json --raw gpurun_out/r06_anat_c2b.npz
step prof_c4 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --profile-json gpurun_out/r06_prof_c4.json
step anat_c4 200 env LMM_AMD_LIB=simgrid_amd/_anat/liblmm_amd.so python scripts/anatomy.py --workload c4 --rounds 30,31,70,71 \
  --product-profile gpurun_out/r06_prof_c4.json --out gpurun_out/r06_c4_round_anatomy.json --raw gpurun_out/r06_anat_c4.npz
step depth 400 python scripts/depth.py --device --systems c4,c2_100,c2_10 --out gpurun_out/r06_depth.json
exit 0
