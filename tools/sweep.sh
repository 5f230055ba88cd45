#!/bin/bash
# Generic A/B sweep on the GPU box.  A recipe file (tools/sweeps/*.txt) holds one
# run per line:  tag | ENV=V ENV2=V2 | command args
# ("bench ..." runs bench.py, "burst ..." tools/burst.py, "pass ..." tools/pass_times.py,
# anything else runs as given).  Every run has its own time limit (LIMIT, default 240 s)
# and the first failure ends the sweep.  The last JSON line of each run is printed
# (value, ms_per_step, and the fields named in FIELDS).
#   bash tools/sweep.sh tools/sweeps/group_test.txt
set -o pipefail
export TMPDIR=/tmp
recipe=$1; name=$(basename "$recipe" .txt)
OUT=gpurun_out/sweep_$name
mkdir -p $OUT
while IFS='|' read -r tag envs cmd; do
  tag=$(echo $tag); [ -z "$tag" ] && continue; case "$tag" in \#*) continue;; esac
  set -- $cmd
  case "$1" in
    bench) shift; set -- python3 -u bench.py --cpu-sample 0 "$@";;
    burst) shift; set -- python3 -u tools/burst.py "$@";;
    pass)  shift; set -- python3 -u tools/pass_times.py "$@";;
  esac
  env FTS_SWEEP=1 $envs timeout -k 10 ${LIMIT:-240} "$@" > $OUT/$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $OUT/$tag.log; exit 1; }
  grep '^{' $OUT/$tag.log | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read() or '{}')
print('$tag', d.get('value', d.get('median')), d.get('ms_per_step', d.get('merged')), *[d.get(f) for f in '${FIELDS:-}'.split()])" 2>/dev/null ||
  tail -1 $OUT/$tag.log | sed "s/^/$tag /"
done < "$recipe"
