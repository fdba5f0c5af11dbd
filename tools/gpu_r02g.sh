#!/bin/bash
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_addon.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "two_ranks or addon or packed" > $O/pytest.log 2>&1; rc=$?; echo rc=$rc >> $O/pytest.log; exit $rc
