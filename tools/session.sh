#!/bin/bash
# One GPU session from a plan file (replaces round 2's one-off *_session.sh
# scripts).  Each plan line is `<name> <timeout-s> <command...>`; `#` starts a
# comment.  Every step runs under its own `timeout -k 10`, writes
# gpurun_out/<tag>/<name>.log, and the session stops at the first step that
# faults, aborts or times out (exit codes other than 0, 1 = test failures,
# 3 = bench device error, 4 = bench frame check).  After the steps, every
# bench JSON line is summarised.
#   tools/session.sh <tag> <plan-file>
# Plan shorthands:
#   bench <args>            python bench.py <args>
#   smoke                   __graft_entry__.smoke()
#   pytest <args>           the GPU test suite (-m gpu -x, 120 s per test)
#   variant <lib> <args>    bench.py against tools/variants/lib_<lib>.so
#   pmc <dir> <ctrs> -- <cmd...>   one rocprofv3 --pmc pass (counters only)
#   stats <dir> -- <cmd...>        rocprofv3 --kernel-trace --stats
#   trace <dir> -- <cmd...>        + --memory-copy-trace; traces kept gzipped (dir must start trace_)
#   setenv VAR VALUE / unsetenv VAR  environment of the following steps
#   pmcsum <key> <kernel> <dir...> [--one]  tools/pmc_traffic.py over pmc dirs of this session
set -u
TAG=$1; PLAN=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
# the pushed library must be this tree's build (rt_build_id); rebuild here if not
python3 - <<'PYEOF' || { echo "stopping: library build failed"; exit 1; }
import os, re, sys
sys.path.insert(0, os.getcwd())
from cpp_cuda_raytracer_dev_amd import _lib, build
want = build.source_id()
got = None
if os.path.exists(_lib.LIB_PATH):
    m = re.search(rb"generated-id:([0-9a-f]{64})", open(_lib.LIB_PATH, "rb").read())
    got = m.group(1).decode() if m else None
print("library build id", (got or "missing")[:16], "tree", want[:16], flush=True)
if got != want:
    print("rebuilding the library for this tree", flush=True)
    build.build_lib()
PYEOF
while read -r name to rest; do
    [ -z "${name:-}" ] && continue
    case $name in \#*) continue ;; esac
    eval "set -- $rest"  # plan lines may quote arguments
    # `setenv VAR VALUE` / `unsetenv VAR`: the environment of the steps that
    # follow (never put `env` after rocprofv3's `--`: the profiled program must
    # be the program itself)
    case $name in
    setenv) export "$to=$1"; echo "== setenv $to=$1"; continue ;;
    unsetenv) unset "$to"; echo "== unsetenv $to"; continue ;;
    esac
    case $1 in
    bench) shift; cmd=(python -u bench.py "$@") ;;
    smoke) cmd=(python -u -c "import __graft_entry__ as g; g.smoke()") ;;
    pytest) shift; cmd=(python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread "$@") ;;
    variant) shift; lib=$1; shift; cmd=(python -u tools/bench_variant.py "tools/variants/lib_$lib.so" "$@") ;;
    pmc) shift; d=$1; shift; ctrs=(); while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
         cmd=(rocprofv3 --pmc "${ctrs[@]}" --output-format csv -d "$OUT/$d" -o run -- "$@") ;;
    pmcsum) shift; k=$1; ks=$2; shift 2; ds=(); one=()
            for d in "$@"; do if [ "$d" = "--one" ]; then one=(--one); else ds+=("$OUT/$d"); fi; done
            cmd=(python3 tools/pmc_traffic.py --out "$OUT/pmc_traffic_$k.json" ${one[@]+"${one[@]}"} "$k" "$ks" "${ds[@]}") ;;
    stats) shift; d=$1; shift; [ "$1" = "--" ] && shift
           cmd=(rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$d" -o run -- "$@") ;;
    trace) shift; d=$1; shift; [ "$1" = "--" ] && shift  # kernel + memory-copy trace, kept (gzipped)
           cmd=(rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/$d" -o run -- "$@") ;;
    *) cmd=("$@") ;;
    esac
    echo "== $name ($to s): ${cmd[*]}"
    t0=$(date +%s)
    timeout -k 10 "$to" "${cmd[@]}" > "$OUT/$name.log" 2>&1 < /dev/null
    rc=$?
    echo "== $name exit $rc ($(( $(date +%s) - t0 )) s)"
    tail -n 3 "$OUT/$name.log" | cut -c1-400
    case $rc in 0|1|3|4) ;; *) echo "stopping: $name exited $rc"; break ;; esac
done < "$PLAN"
python3 tools/bench_summary.py "$OUT"/*.log 2>/dev/null
# gpurun copies gpurun_out/ back only below 64 MiB: drop the per-dispatch
# kernel traces (the stats CSVs stay) and compress the counter CSVs
find "$OUT" -path '*trace_*' -name '*_trace.csv' -exec gzip -f {} \; 2>/dev/null
find "$OUT" -name '*_kernel_trace.csv' -delete 2>/dev/null
find "$OUT" -name '*_counter_collection.csv' -size +1M -exec gzip -f {} \; 2>/dev/null
du -sh "$OUT" 2>/dev/null
echo "session $TAG done"
