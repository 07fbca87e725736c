#!/bin/bash
# Round 4: where the one-wave-per-SIMD bf16 kernel's cycles go against the 8-phase kernel and hipBLASLt at the
# headline stand-in shape (bf16 4-wave: same LDS reads per MFMA as the vendor, higher clock than the 8-phase
# kernel, fewer MFMA per clock). Two PMC passes (8 SQ + GRBM each) over gemm_bench's interleaved rounds, then the
# same two for fp8 (4-wave vs _scaled_mm). Output: gpurun_out/stalls_<dtype>_<pass>/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=8192x4096x14336
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
for d in bf16 fp8; do
  if [ $d = bf16 ]; then V=0,5; else V=5; fi
  for p in 1 2; do
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d gpurun_out/stalls_${d}_$p -o g -- python3 -m dlnetbench_amd.tools.gemm_bench \
      --dtype $d --variants $V --shapes $S --rounds 2 --iters 5 > gpurun_out/stalls_${d}_$p.log 2>&1 || exit $?
  done
done
echo done > gpurun_out/stalls_done.txt
