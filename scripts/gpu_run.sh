#!/bin/bash
# Generic GPU step runner: each argument is "name:limit:command"; steps run in order, each under its
# own time limit, output to gpurun_out/<name>.log; a crash/timeout (rc > 1) stops the script.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; lim=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1; rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
done
exit 0
