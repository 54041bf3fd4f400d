#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03n
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_debug_build.py -m gpu -v --timeout 150 --timeout-method thread > $O/debug_tests.log 2>&1 &&
timeout -k 10 200 ./tools/overlap_bench2 > $O/overlap6.txt 2>&1
echo "rc=$?"
