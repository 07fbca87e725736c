# xgmi release-mode A/B (DLNB_XGMI_RELEASE=vmcnt, the default, vs system, the fallback bench.py takes when the
# exactness pass fails with vmcnt): 2 and 8 ranks sharing GPU 0, staged and zero-copy registered, graph-replayed,
# exactness checked first by xgmi_sweep.sh. Output: gpurun_out/release_ab/*.jsonl.
set -u
mkdir -p gpurun_out/release_ab
for rel in vmcnt system; do
  for W in 2 8; do
    for ex in "" "--registered"; do
      rm -f gpurun_out/xgmi_sweep.jsonl
      DLNB_XGMI_RELEASE=$rel EXTRA="$ex" bash scripts/xgmi_sweep.sh $W uncached 256 "1048576,16777216,67108864" || exit $?
      mv gpurun_out/xgmi_sweep.jsonl gpurun_out/release_ab/${rel}_w${W}${ex:+_reg}.jsonl
    done
  done
done
ls gpurun_out/release_ab
