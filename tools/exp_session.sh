#!/bin/bash
# Experiment session: optional GPU tests (-k filter), then bench.py once per
# line of an argument file (each line: <name> <bench args...>), each under its
# own time limit; stops at the first crash / timeout.
#   tools/exp_session.sh <tag> <pytest -k expr or -> <argfile>
set -u
TAG=$1; KEXPR=$2; ARGS=$3
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -x tools/ubench_pk ] && [ "${UBENCH:-0}" = 1 ]; then
  timeout -k 10 60 tools/ubench_pk > $OUT/ubench.log 2>&1; echo "ubench rc $?"; cat $OUT/ubench.log
fi
if [ "$KEXPR" != "-" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "$KEXPR" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc $rc"; tail -3 $OUT/pytest.log
  [ $rc -le 1 ] || exit $rc
fi
while read -r name rest; do
  [ -z "$name" ] && continue
  case $name in \#*) continue ;; esac
  # "variant:<lib.so> args..." runs bench.py against that build
  cmd="python bench.py"
  case $rest in variant:*) lib=${rest%% *}; cmd="python tools/bench_variant.py ${lib#variant:}"; rest=${rest#* } ;; esac
  timeout -k 10 300 $cmd $rest > $OUT/bench_$name.log 2>&1
  rc=$?
  case $rc in 0|3|4) ;; *) echo "bench $name exited $rc"; tail -5 $OUT/bench_$name.log; exit $rc ;; esac
done < "$ARGS"
python tools/bench_summary.py $OUT/bench_*.log
