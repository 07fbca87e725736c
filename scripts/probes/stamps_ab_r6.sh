# hybrid_3d 2 8 1 on 2 loopback rank threads (eager, sleep compute): kernel counts with task-stamp timers on / off
set -u
mkdir -p gpurun_out/r6x
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 1 0; do
  DLNB_TASK_STAMP_TIMERS=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6x/s$v -o k -- \
    ./build/bin/hybrid_3d tiny_dense_8_bfloat16 2 8 1 tests/data --no-topology --backend loopback --ranks 2 --compute sleep \
    -w 2 -r 5 --quiet --json gpurun_out/r6x/s$v.json > gpurun_out/r6x/s$v.log 2>&1 || exit 1
done
