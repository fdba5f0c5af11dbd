#!/bin/bash
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "chunked or multipass or ref_precision" > $O/pytest.log 2>&1 || exit $?
RT_AMD_REC_SLOT_MAJOR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "chunked or multipass or ref_precision" > $O/pytest_sm.log 2>&1 || exit $?
export OUT=$O/ab CFGS="cornell
spheres --scene spheres --spp 64 --depth 8
cornell8 --scene cornell --width 283
c100k --scene spheres100k --width 2048 --spp 64 --depth 100" ARMS="base
slotmajor RT_AMD_REC_SLOT_MAJOR=1"
bash tools/ab_env.sh || exit $?
python tools/ab_table.py $O/ab > $O/ab_table.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for arm in base slotmajor; do
  E=""; [ $arm = slotmajor ] && E="RT_AMD_REC_SLOT_MAJOR=1"
  env $E timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$O/pmc_w_$arm -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu --no-count > $R/$O/pmc_w_$arm.log 2>&1 || exit $?
done
