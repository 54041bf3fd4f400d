# Build the production library and the KURA_STAMPS diagnostic variant in-tree
# (both travel to the GPU box with gpurun).
set -e
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()"
cd dbs-gym_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
      -DKURA_STAMPS -o libkura_stamps.so kura_kernels.hip
