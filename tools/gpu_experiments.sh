#!/bin/bash
# Round-3 A/B experiments behind profiles/r03/ (one parameterised script; run from the repo root
# on the GPU box). usage: TAG=<out> bash tools/gpu_experiments.sh <experiment>
#   (wpool_ab / wf_ab / wf_prof / wf_pmc: the round-3 walker-pool and wavefront arms, retired with those
#    kernels in round 4 - DESIGN.md §4; their logs stay under profiles/r03/)
#   tail_ab    rank-0 shares N = 1..8 (tools/rank_share.py) under $ARMS env settings -> profiles/r03/tail/
#   variant_ab parity tests (-k $KSEL) on the variant libraries in $VARIANTS, then bench arms
#              (Cornell ref / fp32 unless $CFGS) for the product library and each variant
#   adapt_jump adaptive bench lines (reference defaults) under RT_AMD_ADAPT_JUMP arms   -> profiles/r03/exp2/
#              (the Cornell arms of exp2 ran a variant library, RT_AMD_VARIANT=<name>, built with
#              _build.build_native(variant=..., defines=[...]))
#   sched_r03  rank shares N = 1..8 (SWEEP_TG) under the pool kernel's first-item chunk (Cornell) and
#              min_ready (spheres-500), three repeats; spheres-500 tile-chunks per atomic, two repeats;
#              adaptive Cornell (reference defaults) under first items of 1 / 2     -> profiles/r03/sched/
# $ARMS / $CFGS override the arms and configurations (lines "name ENV=V ..." / "name bench-args").
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
T=${TAG:-exp}
O=gpurun_out/$T
mkdir -p $O
S100K="--scene spheres100k --width 2048 --spp 16 --depth 100"
ab() {  # ab <pytest -k expr> <default CFGS> <default ARMS>
  bash tools/gpu_run.sh $T "pytest:$1" || exit $?
  export OUT=$O/ab CFGS="${CFGS:-$2}" ARMS="${ARMS:-$3}"
  STEPS=3 bash tools/ab_env.sh || exit $?
  python tools/ab_table.py $OUT > $OUT/table.txt
}
case $1 in
  tail_ab)
    echo "${ARMS:-base RT_AMD_TAIL=0}" | while read -r arm envs; do
      [ -z "$arm" ] && continue
      for sc in cornell spheres; do
        env $envs timeout -k 10 200 python tools/rank_share.py $sc > $O/rs_${sc}_${arm}.log 2>&1 || exit $?
      done
    done ;;
  variant_ab)
    for v in $VARIANTS; do
      RT_AMD_VARIANT=$v timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
        -p no:cacheprovider -k "${KSEL:-cornell or pool or brute or config1 or golden or random or full_size or fp32}" \
        > $O/pytest_$v.log 2>&1 || exit $?
    done
    export OUT=$O/ab
    A="base RT_AMD_VARIANT="
    for v in $VARIANTS; do A="$A
$v RT_AMD_VARIANT=$v"; done
    CFGS="${CFGS:-cornell --steps 5
cornellfp32 --precision fp32 --steps 5}" ARMS="$A" STEPS=5 bash tools/ab_env.sh || exit $?
    CFGS="${CFGS:-cornell --steps 5
cornellfp32 --precision fp32 --steps 5}" ARMS="$A" STEPS=5 OUT=$O/ab2 bash tools/ab_env.sh || exit $?
    python tools/ab_table.py $OUT > $OUT/table.txt; python tools/ab_table.py $O/ab2 > $O/ab2/table.txt ;;
  adapt_jump)
    export OUT=$O/ab
    CFGS="${CFGS:-acornell --adaptive
aspheres --scene spheres --spp 64 --depth 8 --adaptive
arain --scene rain --width 1920 --spp 512 --depth 16 --adaptive}" ARMS="${ARMS:-j0 RT_AMD_ADAPT_JUMP=0
j20 RT_AMD_ADAPT_JUMP=20
j50 RT_AMD_ADAPT_JUMP=50
j100 RT_AMD_ADAPT_JUMP=100
j200 RT_AMD_ADAPT_JUMP=200}" STEPS=5 bash tools/ab_env.sh || exit $?
    python tools/ab_table.py $OUT > $OUT/table.txt ;;
  sched_r03)
    for rep in 1 2 3; do
      for tg in 1 2 4 8; do
        SWEEP_TG=$tg SWEEP_VARS="RT_AMD_CHUNK=auto,2,1" timeout -k 10 120 python tools/env_sweep.py cornell >> $O/cornell_chunk.log 2>&1 || exit $?
        SWEEP_TG=$tg SWEEP_VARS="RT_AMD_READY=auto,40" timeout -k 10 120 python tools/env_sweep.py spheres >> $O/spheres_ready.log 2>&1 || exit $?
      done
    done
    for rep in 1 2; do
      for tg in 4 8; do
        SWEEP_TG=$tg SWEEP_VARS="RT_AMD_POOL=auto,1,4" timeout -k 10 120 python tools/env_sweep.py spheres >> $O/spheres_pool.log 2>&1 || exit $?
      done
    done
    OUT=$O/adaptive CFGS="adapt --adaptive" ARMS="base
c1 RT_AMD_CHUNK=1
c2 RT_AMD_CHUNK=2" STEPS=5 bash tools/ab_env.sh || exit $? ;;
  *) echo "unknown experiment $1" >&2; exit 2 ;;
esac
