#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/pmc_pass.sh r03l_k1t && KURA_KERNEL=k1 bash tools/pmc_pass.sh r03l_k1
echo "rc=$?"
