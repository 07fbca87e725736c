# Measured stats tables on one MI355X (dlnetbench_amd.models.measure), one
# model per process, each under its own time limit.
set -u
mkdir -p gpurun_out model_stats_measured
for spec in vit_b:bfloat16 vit_l:bfloat16 vit_h:bfloat16 vit_h:float8 gpt2_l:bfloat16 gpt2_xl:bfloat16 \
            llama3_8b:bfloat16 llama3_8b:float8 minerva_7b:bfloat16 llama3_70b:bfloat16 mixtral_8x7b:bfloat16; do
  m=${spec%%:*}; dt=${spec##*:}
  timeout -k 10 240 python -m dlnetbench_amd.models.measure $m --batch_size 16 --dtype $dt --out model_stats_measured \
    >> gpurun_out/measure.log 2>&1
  rc=$?
  echo "$spec rc=$rc" >> gpurun_out/measure_steps.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
cp -r model_stats_measured gpurun_out/
