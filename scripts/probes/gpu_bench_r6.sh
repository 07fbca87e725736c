set -o pipefail
mkdir -p gpurun_out/r6c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c/prof_gw -o gw -- ./build/bin/dp vit_h_32_float8 8 . --no-topology -w 5 -r 10 --compute gemm-work --backend rccl --graph --quiet --json gpurun_out/r6c/gw.json > gpurun_out/r6c/gw.log 2>&1 &&
timeout -k 10 900 python -u bench.py > gpurun_out/r6c/bench.log 2> gpurun_out/r6c/bench.err
