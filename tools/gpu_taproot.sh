#!/bin/bash
# GPU check of the Taproot path: the taproot tests first (fast fail), then the whole -m gpu suite.
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_taproot_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_taproot.log 2>&1 || { tail -40 $O/pytest_taproot.log; exit 1; }
tail -3 $O/pytest_taproot.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 2; }
tail -3 $O/pytest_gpu.log
