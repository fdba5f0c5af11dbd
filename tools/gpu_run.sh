#!/bin/bash
# One parameterised GPU session runner (replaces the per-session gpu_*.sh scripts).
# usage: bash tools/gpu_run.sh <tag> <step> [<step> ...]     (from $GRAFT_REPO_ROOT on the box)
# steps:
#   pytest            the -m gpu suite (per-test thread timeout)
#   pytest:<expr>     the -m gpu suite restricted by -k <expr>
#   bench             the default bench line (N=1 headline, CPU leg + parity)
#   bench4            Cornell ref / spheres-500 / rain 1080p spp512 / spheres-100k spp16 (no CPU leg)
#   fp32              Cornell in fp32 mode
#   adaptive          Cornell 800^2 spp256 with the reference's adaptive defaults
#   config5           BASELINE config 5 (spheres-100k 4096^2 spp1024 depth 100)
#   prof              bench under rocprofv3 --kernel-trace --stats (csv)
#   valu / traffic    the VALU / HBM counter passes of the bench configs + fp32 + adaptive (separate --pmc runs)
#   valu5 / traffic5  the same for BASELINE config 5 (spheres-100k 4096^2 spp1024 depth 100, 32 passes)
#   rankshare         tools/rank_share.py: every tile group of N = 2, 4, 8 (max / min / mean) + RCCL gather + unpack
#   sections          tools/profile_sections.py (section timers of the chunked / sequential kernels)
#   poolsections      the same for the pool kernel (variant library 'poolprof': RT_POOL_PROF=1, RT_POOL_K=146)
#   countexact        tools/count_exact.py (exact tests per ray / per wave-trip)
#   single            bench.py --single-process (rt_camera_render_multi): N=1, and N=4 on device 0 repeated
#   bench:<args>      one extra bench line with <args> (underscores become spaces)
#   ab                runtime-knob A/B (tools/ab_env.sh) over $CFGS x $ARMS (set by the caller:
#                     lines "tag bench-args" / "arm ENV=V ..."), table in $O/ab/table.txt
#   abvar             library-variant A/B: $ARMS lines "arm variant" (RT_AMD_VARIANT, '-' = default lib)
# Every GPU step runs under its own time limit; the first failing step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $R/$O
cd $R
B="python bench.py --no-cpu"
CFGS4=("" "--scene spheres --spp 64 --depth 8" "--scene rain --width 1920 --spp 512 --depth 16" \
       "--scene spheres100k --width 4096 --spp 16 --depth 100")
CFG5="--scene spheres100k --width 4096 --spp 1024 --depth 100"
run() {  # run <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$(date +%T) $log rc=$rc" >> $O/steps.txt
  return $rc
}
for step in "$@"; do
  case $step in
    pytest) run 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit $? ;;
    pytest:*) run 900 pytest_k.log python -u -m pytest tests -m gpu -x -v -k "${step#pytest:}" --timeout 200 --timeout-method thread -p no:cacheprovider || exit $? ;;
    bench) run 300 bench_default.log python bench.py || exit $? ;;
    bench4)
      run 200 b_cornell.log $B --steps 5 --warmup 1 || exit $?
      run 200 b_spheres.log $B ${CFGS4[1]} --steps 5 --warmup 1 || exit $?
      run 200 b_rain.log $B ${CFGS4[2]} --steps 3 --warmup 1 || exit $?
      run 300 b_100k.log $B ${CFGS4[3]} --steps 2 --warmup 1 || exit $? ;;
    fp32) run 200 b_cornell_fp32.log $B --precision fp32 --steps 5 --warmup 1 || exit $? ;;
    adaptive) run 300 b_adaptive.log $B --adaptive --steps 3 --warmup 1 || exit $? ;;
    config5) run 600 b_config5.log $B $CFG5 --steps 1 --warmup 0 --no-count || exit $? ;;
    single)  # one process, all N GPUs through rt_camera_render_multi (device 0 repeated on a 1-GPU box)
      run 300 b_single1.log python bench.py --single-process --gpus 1 --no-cpu --steps 10 || exit $?
      run 300 b_single4.log python bench.py --single-process --gpus 4 --devices 0,0,0,0 --no-cpu --steps 10 || exit $? ;;
    bench:*) a=${step#bench:}; run 300 b_extra_$(echo $a | tr -c 'a-z0-9' _ | cut -c1-40).log $B ${a//_/ } || exit $? ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run \
        --output-format csv -- python3 $R/bench.py --no-cpu > $R/$O/prof.log 2>&1) || exit $? ;;
    valu) VALU_DIR=$O/valu bash tools/pmc_valu.sh "${CFGS4[@]}" "--precision fp32" "--adaptive" || exit $? ;;
    valu5) VALU_DIR=$O/valu5 bash tools/pmc_valu.sh "$CFG5" || exit $? ;;
    traffic) TRAFFIC_DIR=$O/traffic bash tools/pmc_traffic.sh "${CFGS4[@]}" "--precision fp32" "--adaptive" || exit $? ;;
    traffic5) TRAFFIC_DIR=$O/traffic5 bash tools/pmc_traffic.sh "$CFG5" || exit $? ;;
    rankshare) run 400 rank_share.log python tools/rank_share.py cornell spheres rain || exit $? ;;
    sections) run 300 sections.log python tools/profile_sections.py || exit $? ;;
    sections:*) run 300 sections_${step#sections:}.log python tools/profile_sections.py ${step#sections:} || exit $? ;;
    ab) OUT=$O/ab bash tools/ab_env.sh || exit $?; python tools/ab_table.py $O/ab > $O/ab/table.txt ;;
    abvar)
      mkdir -p $O/ab
      echo "$CFGS" | while read -r tag args; do
        [ -z "$tag" ] && continue
        echo "$ARMS" | while read -r arm var; do
          [ -z "$arm" ] && continue
          if [ "$var" = "-" ]; then vv=""; else vv=$var; fi
          RT_AMD_VARIANT=$vv run ${TLIM:-200} ab/${tag}_${arm}.log python bench.py --steps ${STEPS:-5} --warmup 1 \
            --no-cpu --no-count --no-parity $args || exit $?
        done || exit $?
      done || exit $?
      python tools/ab_table.py $O/ab > $O/ab/table.txt ;;
    poolsections) RT_AMD_VARIANT=poolprof run 300 sections_pool.log python tools/profile_sections.py cornell || exit $? ;;
    countexact) run 300 count_exact.log python tools/count_exact.py || exit $? ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
exit 0
