#!/bin/bash
# Same-box A/B/... of library builds, interleaved R rounds of `bench.py --no-cpu-baseline $BARGS`.
#   LIBS="A=path/libA.so B=path/libB.so ..." (default: A = csrc/build/ab/libA.so, made by scripts/build_ab.sh
#   <ref>, and B = the tree's own library)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
LIBS=${LIBS:-"A=$PWD/endoscopy-image-classification_amd/csrc/build/ab/libA.so B=$PWD/endoscopy-image-classification_amd/endossl/lib/libendossl_hip.so"}
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'], round(d.get('roofline', {}).get('mean_launch_ms', 0), 4))"; }
for r in $(seq ${R:-3}); do
  line="round $r"
  for kv in $LIBS; do
    k=${kv%%=*}; lib=${kv#*=}
    ENDOSSL_LIB=$lib timeout -k 10 ${LIM:-240} python -u bench.py --no-cpu-baseline ${BARGS} > "$OUT/abl_${k}$r.log" 2>&1 || exit 1
    line="$line  $k $(ms $OUT/abl_${k}$r.log)"
  done
  echo "$line"
done
