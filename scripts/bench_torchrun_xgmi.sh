# The N>1 bench path (torchrun rendezvous, multi-rank FSDP, rank-0 JSON) on a
# 1-GPU box: N ranks share GPU 0 through the xgmi backend (RCCL refuses two
# ranks on one device). Collectives are local-HBM copies, so only the
# plumbing and the compute-floor accounting are meaningful here.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=120
for n in 2 4; do
  devs=$(python3 -c "print(','.join(['0']*$n))")
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29700 + n)) bench.py --gpus $n --steps 2 --warmup 1 --backend xgmi --devices $devs \
    > gpurun_out/bench_xgmi_n$n.log 2> gpurun_out/bench_xgmi_n$n.err
  rc=$?
  echo "n=$n rc=$rc $(grep '^{' gpurun_out/bench_xgmi_n$n.log | head -1 | cut -c1-400)" >> gpurun_out/bench_xgmi_steps.log
  [ $rc -eq 0 ] || exit $rc
done
