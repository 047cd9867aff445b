#!/bin/bash
# GPU box: one parameterised batch of steps (replaces round 4's one-off tools/r04*.sh scripts).
#   bash tools/gpu_batch.sh <tag> <step> [<step> ...]
# Steps run in order, each under its own time limit; the batch stops at the first failing step (and
# so never starts another GPU step after a crash, a fault or a time limit).  Outputs land in
# gpurun_out/<tag>_*.
#   tests                      the whole GPU suite                 -> <tag>_gpu_tests.log
#   test:<pytest args>         a selection (eval'd: quote a -k expression inside it):
#                              "test:tests/test_gpu_ops.py -k 'peg or vq'" -> <tag>_tests<i>.log
#   smoke                      __graft_entry__.smoke()             -> <tag>_smoke.log
#   bench[:<bench.py args>]    bench.py                            -> <tag>_bench.log
#   prof                       tools/prof_bench.sh <tag>: bench + rocprof kernel summary, grid, streams,
#                              timeline, sequence                  -> <tag>_kernel_stats.txt ...
#   abenv:<A>|<B>[|reps]       same-box interleaved env A/B of bench.py (A, B = "VAR=x VAR2=y")
#                                                                  -> <tag>_ab_env.log (+ means)
#   cmd:<command>              anything else (600 s limit)         -> <tag>_cmd<i>.log
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=$1
shift
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%:*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*:}
  echo "== step $i: $step"
  case $name in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread \
        > gpurun_out/${tag}_gpu_tests.log 2>&1
      rc=$?; tail -3 gpurun_out/${tag}_gpu_tests.log ;;
    test)
      eval timeout -k 10 900 python -u -m pytest -m gpu -x -v -rP --timeout 300 --timeout-method thread "$arg" \
        > gpurun_out/${tag}_tests${i}.log 2>&1
      rc=$?; tail -3 gpurun_out/${tag}_tests${i}.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/${tag}_smoke.log ;;
    bench)
      timeout -k 10 400 python -u bench.py $arg > gpurun_out/${tag}_bench.log 2>&1
      rc=$?; tail -1 gpurun_out/${tag}_bench.log ;;
    prof)
      bash tools/prof_bench.sh ${tag}
      rc=$?; grep -E "TOTAL" gpurun_out/${tag}_kernel_stats.txt | head -3 ;;
    abenv)
      IFS='|' read -r ea eb reps <<< "$arg"
      reps=${reps:-3}
      out=gpurun_out/${tag}_ab_env.log
      : > $out
      rc=0
      for r in $(seq $reps); do
        for e in "$ea" "$eb"; do
          line=$(env $e timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-precise 2>>gpurun_out/${tag}_ab_env.err | tail -1)
          rc=$?
          [ $rc -ne 0 ] && break 2
          echo "$e | $line" >> $out
        done
      done
      python - "$out" <<'PY'
import json, sys
res = {}
for line in open(sys.argv[1]):
    e, _, js = line.partition(' | ')
    try:
        d = json.loads(js)
    except ValueError:
        continue
    res.setdefault(e, []).append((d['value'], d['ms_per_step'], (d.get('vit_forward') or {}).get('ms')))
for e, v in res.items():
    n = len(v)
    print(f"{e}: pairs/s {[x[0] for x in v]} mean {sum(x[0] for x in v) / n:.2f}; "
          f"ms/step mean {sum(x[1] for x in v) / n:.3f}")
PY
      ;;
    cmd)
      timeout -k 10 600 bash -c "$arg" > gpurun_out/${tag}_cmd${i}.log 2>&1
      rc=$?; tail -5 gpurun_out/${tag}_cmd${i}.log ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  echo "== step $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
