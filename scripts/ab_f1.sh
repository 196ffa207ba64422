cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export ENDOSSL_LIB=$GRAFT_REPO_ROOT/build/ab/HEAD/libendossl_hip.so; else unset ENDOSSL_LIB; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v$r.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab_$v$r.log | python -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
