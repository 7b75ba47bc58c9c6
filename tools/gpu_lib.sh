# Shared helpers for the GPU-box scripts (sourced).  Every GPU step runs under
# its own time limit; a step that ends in a fault, abort, segfault, time limit
# or hang (any status other than 0 / 1) ends the whole script, so nothing more
# touches the GPU after trouble.  Status 1 (a failed test, a Python error) is
# recorded and the script goes on.
set -o pipefail
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "[$(date +%T)] $name: $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "[$(date +%T)] $name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        tail -5 "$OUT/$name.err"
        exit $rc
    fi
    return 0
}
pmc() {  # pmc NAME COUNTER CMD...  (one counter group per pass, killed hard if it hangs)
    local name=$1 ctr=$2
    shift 2
    echo "[$(date +%T)] pmc $name: $ctr"
    timeout -s KILL 240 rocprofv3 --pmc "$ctr" -d "$OUT/$name" -o "$name" --output-format csv -- "$@" \
        > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "[$(date +%T)] pmc $name rc=$rc"
    if [ $rc -ne 0 ]; then echo "stopping after pmc $name (rc=$rc)"; exit $rc; fi
}
export TMPDIR=/tmp
