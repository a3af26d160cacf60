#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment gpu_r0*.sh
# scripts of rounds 3-4).  Each STEP runs under its own time limit, writes
# gpurun_out/<TAG>/<n>_<step>.log and prints its tail; the first failure ends
# the run (no retries).
#
# usage (repo root, on the GPU box): bash scripts/gpu_run.sh TAG STEP [STEP ...]
#   smoke                   __graft_entry__.smoke()
#   suite[:ARGS]            pytest -m gpu over tests/ (ARGS: the files / pytest args instead)
#   bench[:ARGS]            bench.py --steps 20 --warmup 5 ARGS (the driver's shape)
#   ab:V1,V2:REPS[:ARGS]    alternating bench lines of abvar/V1.so, abvar/V2.so, ...
#                           (scripts/build_variant.sh builds them; "prod" = this tree's library)
#   parity:V[:ARGS]         the FFT parity + fuzz tests with abvar/V.so in place
#   fuzz:SEED0,CASES,NORM[,FAMILY]  seeded fuzz campaign (tests/test_gpu_fuzz.py; FAMILY: default, lds)
#   trace[:ARGS]            tools/fft32r_trace phase timeline (default 4001 32768)
#   vtrace:V[:ARGS]         the same tool built from variant V's source (abvar/V.trace)
#   prof[:ARGS]             rocprofv3 --kernel-trace --stats of a bench line + the
#                           exclusive launches from its trace
#   pmc[:ARGS]              FETCH_SIZE / WRITE_SIZE / VALU-instruction passes (one
#                           rocprofv3 --pmc run each) + pmc_summary.json
#   pmcre:REGEX[:ARGS]      FETCH_SIZE / WRITE_SIZE passes over the kernels matching REGEX
#   pmcx:C1,C2,..:REGEX[:ARGS]  one --pmc pass of those counters (per-block limits apply)
#   traffic:NTAPS:SPL:KERNEL:SEG[:ARGS]  bench.py's PMC sidecar (traffic.json) for one bench line
#   tool:NAME[:ARGS]        audio-fir-filter_amd/tools/NAME (a built development tool)
#   dropin[:ARGS]           tests/cpp/dropin_bench
#   dropin_nosdma[:ARGS]    the same with HSA_ENABLE_SDMA=0 (copies by blit kernels)
#   vdropin:V[:ARGS]        the same over variant V's library
#   dropintrace[:V[:ARGS]]  kernel + memory-copy trace of the pinned drop-in (copy_overlap.py)
#   gpus2[:ARGS]            bench.py --gpus 2 rehearsal on one device (gloo)
# Words in ARGS are separated by spaces (quote the whole STEP).
set -u -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:?tag}; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
N=0
run() { # name timeout cmd...
    local name=$1 t=$2; shift 2
    N=$((N + 1))
    local log="$OUT/${N}_$name.log"
    echo "== $N $name ($(date +%T)): $*" | cut -c1-300
    timeout -k 10 "$t" "$@" > "$log" 2>&1
    local rc=$?
    tail -4 "$log" | cut -c1-3000
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$log"; exit $rc; fi
}
brief() { # the bench line's headline fields
    python3 -c 'import json,sys
for l in sys.stdin:
    if l.startswith("{"):
        d=json.loads(l); r=d["roofline"]; p=d.get("parity",{})
        print(d["value"], d["ms_per_step"], r["kernel_ms"], r["frac"], p.get("rms_vs_longdouble"), p.get("max_ulp"))'
}
LIB=audio-fir-filter_amd/liblcfir.so
HERE_ID=$(bash audio-fir-filter_amd/src_hash.sh)
# a variant must be built on this tree (scripts/build_variant.sh stamps
# abvar/V.base with its base tree's build id); checked for every variant of a
# step before anything runs
check_variant() {
    local v=$1 want
    [ "$v" = prod ] && return 0
    [ -f "abvar/$v.so" ] || { echo "!! variant $v: abvar/$v.so missing"; exit 3; }
    want=$(sed -n 's/.*base_build_id=\([0-9a-f]*\).*/\1/p' "abvar/$v.base" 2>/dev/null)
    if [ "$want" != "$HERE_ID" ]; then
        echo "!! variant $v was built on tree ${want:-<unstamped>}, this tree is $HERE_ID: rebuild it (scripts/build_variant.sh)"
        exit 3
    fi
}
for S in "$@"; do # refuse stale variants before the first step runs
    k=${S%%:*}; r=""; [ "$k" != "$S" ] && r=${S#*:}
    case $k in
    ab) vl=${r%%:*}; for v in ${vl//,/ }; do check_variant "$v"; done ;;
    parity|vtrace|vdropin) check_variant "${r%%:*}" ;;
    dropintrace) v=${r%%:*}; check_variant "${v:-prod}" ;;
    esac
done
cp "$LIB" /tmp/liblcfir_prod.so
restore() { cp /tmp/liblcfir_prod.so "$LIB"; }
trap restore EXIT
for S in "$@"; do
    kind=${S%%:*}
    rest=""; [ "$kind" != "$S" ] && rest=${S#*:}
    case $kind in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    suite) run suite 1500 python -u -m pytest ${rest:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench) run bench 400 python bench.py --steps 20 --warmup 5 $rest ;;
    ab)
        vs=${rest%%:*}; r2=${rest#*:}; reps=${r2%%:*}; args=""; [ "$r2" != "$reps" ] && args=${r2#*:}
        for rep in $(seq 1 "$reps"); do
            for v in ${vs//,/ }; do
                if [ "$v" = prod ]; then restore; else cp "abvar/$v.so" "$LIB"; fi
                N=$((N + 1)); log="$OUT/${N}_ab_${v}_$rep.log"
                timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ingest $args > "$log" 2>&1 \
                    || { echo "!! ab $v failed"; tail -20 "$log"; exit 1; }
                echo "$v rep$rep $(brief < "$log") [$args]" | tee -a "$OUT/ab.txt"
            done
        done
        restore ;;
    parity)
        v=${rest%%:*}; args=""; [ "$v" != "$rest" ] && args=${rest#*:}
        cp "abvar/$v.so" "$LIB"
        run "parity_$v" 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
            tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_baseline_configs.py $args
        restore ;;
    fuzz)
        IFS=, read -r s0 nc nn fam <<< "$rest"
        LCFIR_FUZZ_SEED0=$s0 LCFIR_FUZZ_CASES=$nc LCFIR_FUZZ_NORM_CASES=$nn LCFIR_FUZZ_FAMILY=${fam:-default} \
            run fuzz 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -q -p no:cacheprovider \
            --timeout 120 --timeout-method thread ;;
    trace) run trace 120 audio-fir-filter_amd/tools/fft32r_trace ${rest:-4001 32768} ;;
    vtrace) # vtrace:V[:ARGS] -- the phase trace of variant V (abvar/V.trace)
        v=${rest%%:*}; args=""; [ "$v" != "$rest" ] && args=${rest#*:}
        run "trace_$v" 120 "abvar/$v.trace" ${args:-4001 32768} ;;
    prof)
        # run() in this shell (not a subshell), so the step counter advances
        d="$OUT/prof$((N + 1))"
        cd /tmp; export TMPDIR=/tmp
        run prof 600 rocprofv3 --kernel-trace --stats -f csv -d "$d" -o bench -- \
            python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-ingest $rest
        cd "$ROOT"
        python3 scripts/trace_exclusive.py "$d/bench_kernel_trace.csv" > "$d/exclusive_from_trace.json"
        head -c 600 "$d/exclusive_from_trace.json"; echo ;;
    pmc|pmcre)
        # pmcre:REGEX[:ARGS] -- the kernels matching REGEX (default 'fir_'), traffic passes only
        re='fir_'; passes=(FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64")
        if [ "$kind" = pmcre ]; then
            re=${rest%%:*}; r2=""; [ "$re" != "$rest" ] && r2=${rest#*:}; rest=$r2; passes=(FETCH_SIZE WRITE_SIZE)
        fi
        d="$OUT/$kind$((N + 1))"; i=0
        cd /tmp; export TMPDIR=/tmp
        for c in "${passes[@]}"; do
            i=$((i + 1))
            run "${kind}_$i" 300 rocprofv3 --pmc $c --kernel-include-regex "$re" -f csv \
                -d "$d/p_$i" -o pmc -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
                --no-parity --no-ingest $rest
        done
        cd "$ROOT"
        echo "$rest" > "$d/args.txt"
        python3 scripts/pmc_summary.py "$d" --json "$d/pmc_summary.json" > /dev/null && echo "pmc summary ok: $d" ;;
    pmcx) # pmcx:COUNTERS:REGEX[:ARGS] -- one --pmc pass of the given counters (comma-separated;
        # within rocprofv3's per-block limits) over the kernels matching REGEX
        IFS=: read -r cl re targs <<< "$rest"
        d="$OUT/pmcx$((N + 1))"
        cd /tmp; export TMPDIR=/tmp
        run pmcx 300 rocprofv3 --pmc ${cl//,/ } --kernel-include-regex "$re" -f csv -d "$d/p_1" -o pmc -- \
            python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-ingest ${targs:-}
        cd "$ROOT"
        python3 scripts/pmc_summary.py "$d" --json "$d/pmc_summary.json" > /dev/null && cat "$d/pmc_summary.json" ;;
    traffic) # traffic:NTAPS:SAMPLES_PER_LAUNCH:KERNEL:SEG_LEN[:ARGS] -- the bench's PMC sidecar
        # (profiles/traffic_*.json: FETCH_SIZE, WRITE_SIZE, f64 VALU passes of the
        # bench line ARGS names, scripts/make_traffic_json.py over their summary)
        IFS=: read -r nt spl kern seg targs <<< "$rest"
        d="$OUT/traffic$((N + 1))"; i=0
        cd /tmp; export TMPDIR=/tmp
        for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64"; do
            i=$((i + 1))
            run "traffic_$i" 300 rocprofv3 --pmc $c --kernel-include-regex "$kern" -f csv -d "$d/p_$i" -o pmc -- \
                python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-ingest --ntaps "$nt" ${targs:-}
        done
        cd "$ROOT"
        python3 scripts/pmc_summary.py "$d" --json "$d/pmc_summary.json" > /dev/null &&
        python3 scripts/make_traffic_json.py "$d/pmc_summary.json" "$d/traffic.json" --method fft --ntaps "$nt" \
            --samples-per-launch "$spl" --kernel "$kern" --seg-len "$seg" && cat "$d/traffic.json" ;;
    tool) # tool:NAME[:ARGS] -- a development tool under audio-fir-filter_amd/tools
        t=${rest%%:*}; args=""; [ "$t" != "$rest" ] && args=${rest#*:}
        run "tool_$t" 300 "audio-fir-filter_amd/tools/$t" $args ;;
    dropin) run dropin 600 tests/cpp/dropin_bench ${rest:---threads 1,16,ref --reps 3} ;;
    dropin_nosdma) HSA_ENABLE_SDMA=0 run dropin_nosdma 600 tests/cpp/dropin_bench ${rest:---threads 1,16,ref --reps 3} ;;
    vdropin) # vdropin:V[:ARGS] -- tests/cpp/dropin_bench over variant V's library
        v=${rest%%:*}; args=""; [ "$v" != "$rest" ] && args=${rest#*:}
        cp "abvar/$v.so" "$LIB"
        run "dropin_$v" 600 tests/cpp/dropin_bench ${args:---threads 1,16,ref --reps 3}
        restore ;;
    dropintrace) # dropintrace[:V[:ARGS]] -- kernel + memory-copy trace of the pinned 16-thread drop-in
        # (V: a variant library, default the product), then scripts/copy_overlap.py over it
        v=${rest%%:*}; args=""; [ "$v" != "$rest" ] && args=${rest#*:}; v=${v:-prod}
        [ "$v" = prod ] || cp "abvar/$v.so" "$LIB"
        d="$OUT/dropintrace_$v"
        cd /tmp; export TMPDIR=/tmp
        run "dropintrace_$v" 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace -f csv -d "$d" -o di -- \
            "$ROOT/tests/cpp/dropin_bench" ${args:---threads 16 --reps 1 --modes pinned}
        cd "$ROOT"; restore
        python3 scripts/copy_overlap.py "$d" | tee "$d/overlap.txt" ;;
    gpus2) LCFIR_BENCH_SHARE_DEVICE=1 run gpus2 400 python bench.py --gpus 2 --steps 10 --warmup 2 $rest ;;
    *) echo "unknown step $S"; exit 2 ;;
    esac
done
echo "== done"
