# Run GPU pytest steps in order; a step that fails its tests (rc 1) does not stop the next one, any other
# status (a time limit, an abort, a fault) ends the script there.
# usage: bash scripts/probes/gpu_steps.sh OUTDIR "LIMIT_S LOGNAME PYTEST_ARGS..." ...  ('+' in an arg: a space)
out=$1; shift
mkdir -p "$out"
final=0
for step in "$@"; do
  set -- $step
  lim=$1; log=$2; shift 2
  args=()
  for a in "$@"; do args+=("${a//+/ }"); done  # '+' stands for a space (pytest -k expressions)
  timeout -k 10 "$lim" python -u -m pytest "${args[@]}" -v --timeout-method thread > "$out/$log" 2>&1
  rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && final=$rc
done
exit $final
