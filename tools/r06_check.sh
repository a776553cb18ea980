#!/bin/bash
# round 6: GPU suite + smoke + bench on the current tree
#   bash tools/r06_check.sh <tag> [extra pytest args]
set -o pipefail
R=gpurun_out/$1; mkdir -p $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests ${@:2} \
  > $R/gpu_tests.log 2>&1; rc=$?
tail -n 3 $R/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1 || exit 1
tail -n 1 $R/smoke.log
timeout -k 10 300 python -u bench.py > $R/bench.json 2> $R/bench.err || exit 1
python3 -c "import json;d=json.load(open('$R/bench.json'));print(json.dumps(d['summary']))"
