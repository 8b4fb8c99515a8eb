# Run GPU steps in order on the gpurun box; stop at the first step that did not end normally.
#   bash tools/gpu_steps.sh <name>:<seconds>:<command> ...
# A step "ends normally" with exit 0, or exit 1 for a pytest step (test failures, no crash).  A timeout (124/137),
# abort (134), segfault (139) or any other code ends the script there.
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "[gpu_steps] $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [[ "$cmd" == *pytest* ]]; }; then
    echo "[gpu_steps] stopping after $name"
    exit $rc
  fi
done
