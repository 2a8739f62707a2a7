#!/bin/bash
# Round 5: C2 round-loop cadence knobs re-swept on the final code (same box): compaction cadence / threshold, the
# alive-constraint list cadence, rounds queued per poll, saturation waves per ready constraint.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
line() {  # line <tag> <env...> -- <bench args>
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --dropin-steps 0 \
    > gpurun_out/kn_$tag.json 2> gpurun_out/kn_$tag.log; local rc=$?
  if [ $rc -ne 0 ]; then echo "STOP $tag rc=$rc"; tail -n 20 gpurun_out/kn_$tag.log; exit $rc; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/kn_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'])"
}
if [ "$1" = "7" ]; then  # (a build with kUSeg = 2048)
for pass in a b; do
line u7_1024_$pass LMMHIP_UPDQ_BLOCKS=1024 --
line u7_768_$pass LMMHIP_UPDQ_BLOCKS=768 --
line u7_512_$pass LMMHIP_UPDQ_BLOCKS=512 --
line u7_512s1024_$pass LMMHIP_UPDQ_BLOCKS=512 LMMHIP_SAT_BLOCKS=1024 --
line st_u7_1024_$pass LMMHIP_UPDQ_BLOCKS=1024 -- --variant stress
line st_u7_512_$pass LMMHIP_UPDQ_BLOCKS=512 -- --variant stress
done
echo done
exit 0
fi
if [ "$1" = "6" ]; then
for pass in a b; do
line u6base_$pass LMMHIP_UPDQ_BLOCKS=1024 --
line u6s1280_$pass LMMHIP_UPDQ_BLOCKS=1024 LMMHIP_SAT_BLOCKS=1280 --
line u6s1536_$pass LMMHIP_UPDQ_BLOCKS=1024 LMMHIP_SAT_BLOCKS=1536 --
line u6s2048_$pass LMMHIP_UPDQ_BLOCKS=1024 LMMHIP_SAT_BLOCKS=2048 --
line st_u6s1280_$pass LMMHIP_UPDQ_BLOCKS=1024 LMMHIP_SAT_BLOCKS=1280 -- --variant stress
line st_u6s1536_$pass LMMHIP_UPDQ_BLOCKS=1024 LMMHIP_SAT_BLOCKS=1536 -- --variant stress
done
echo done
exit 0
fi
if [ "$1" = "5" ]; then
for pass in a b; do
line base5_$pass LMMHIP_X=0 --
line uq1024_$pass LMMHIP_UPDQ_BLOCKS=1024 --
line uq1024s768_$pass LMMHIP_UPDQ_BLOCKS=1024 LMMHIP_SAT_BLOCKS=768 --
line uq1024s1280_$pass LMMHIP_UPDQ_BLOCKS=1024 LMMHIP_SAT_BLOCKS=1280 --
line st_base5_$pass LMMHIP_X=0 -- --variant stress
line st_uq1024_$pass LMMHIP_UPDQ_BLOCKS=1024 -- --variant stress
done
echo done
exit 0
fi
if [ "$1" = "4" ]; then
for pass in a b; do
line base4_$pass LMMHIP_X=0 --
line sb768_$pass LMMHIP_SAT_BLOCKS=768 --
line sb1024_$pass LMMHIP_SAT_BLOCKS=1024 --
line sb1280_$pass LMMHIP_SAT_BLOCKS=1280 --
line sb1536_$pass LMMHIP_SAT_BLOCKS=1536 --
line st_base4_$pass LMMHIP_X=0 -- --variant stress
line st_sb1024_$pass LMMHIP_SAT_BLOCKS=1024 -- --variant stress
line st_sb768_$pass LMMHIP_SAT_BLOCKS=768 -- --variant stress
done
echo done
exit 0
fi
if [ "$1" = "3" ]; then
for pass in a b; do
line base3_$pass LMMHIP_X=0 --
line sb512_$pass LMMHIP_SAT_BLOCKS=512 --
line sb1024_$pass LMMHIP_SAT_BLOCKS=1024 --
line sb2048_$pass LMMHIP_SAT_BLOCKS=2048 --
line cmp40_$pass LMMHIP_COMPACT_EVERY=40 --
line cmp56_$pass LMMHIP_COMPACT_EVERY=56 --
done
echo done
exit 0
fi
if [ "$1" = "2" ]; then
for pass in a b; do
line base_$pass LMMHIP_X=0 --
line cmp48_$pass LMMHIP_COMPACT_EVERY=48 --
line cmp64_$pass LMMHIP_COMPACT_EVERY=64 --
line cmp96_$pass LMMHIP_COMPACT_EVERY=96 --
line cmp48c32_$pass LMMHIP_COMPACT_EVERY=48 LMMHIP_CHUNK_MAX=32 --
line cmp64c32_$pass LMMHIP_COMPACT_EVERY=64 LMMHIP_CHUNK_MAX=32 --
line st_base_$pass LMMHIP_X=0 -- --variant stress
line st_cmp48_$pass LMMHIP_COMPACT_EVERY=48 -- --variant stress
line st_cmp64_$pass LMMHIP_COMPACT_EVERY=64 -- --variant stress
done
echo done
exit 0
fi
for pass in a b; do
line base_$pass LMMHIP_X=0 --
line cmp16_$pass LMMHIP_COMPACT_EVERY=16 --
line cmp48_$pass LMMHIP_COMPACT_EVERY=48 --
line pct60_$pass LMMHIP_COMPACT_PCT=60 --
line pct90_$pass LMMHIP_COMPACT_PCT=90 --
line cl4_$pass LMMHIP_CLIST_EVERY=4 --
line cl16_$pass LMMHIP_CLIST_EVERY=16 --
line ch32_$pass LMMHIP_CHUNK_MAX=32 --
line sk1_$pass LMMHIP_SAT_WAVES=1 --
line sk4_$pass LMMHIP_SAT_WAVES=4 --
done
echo done
