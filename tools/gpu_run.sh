#!/bin/bash
# One gpurun call, parameterised (replaces the per-run one-off scripts, whose
# records now live beside their results under profiles/runs/).
# Usage (on the GPU box, from the repo root):
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]
# Steps, run in order, each under its own time limit; the first failure ends
# the call (no GPU step runs after a failed or timed-out one):
#   pytest         the -m gpu suite             -> $O/pytest.log
#   pytest:<expr>  the -m gpu suite, -k <expr>  -> $O/pytest.log
#   smoke          __graft_entry__.smoke()      -> $O/smoke.log
#   c<N>           bench.py --config N           -> $O/bench_c<N>.log (N = 0..4)
#   c<N>full       bench.py --config N --full-parity -> $O/bench_c<N>full.log
#   trace<N>       rocprofv3 --kernel-trace --stats of bench configs[N] -> $O/trace_c<N>/
#   pmc<N>         tools/pmc.sh passes for configs[N] -> gpurun_out/pmc_<tag>_c<N>/
#   split          tools/split_bench.py --gb 20  -> $O/split_bench.log
#   exp:<script>   any tools/<script> with TSG_LIB_VARIANT=exp (A/B runs)
# Extra bench.py arguments for every bench step: BENCH_ARGS="--steps 10".
set -o pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
summ() {  # the bench line's headline fields
  python3 - "$1" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
r = d.get("roofline") or {}
out = dict(value=d["value"], ms=d["ms_per_step"], frac=r.get("frac"), scan_ms=r.get("avg_launch_ms"),
           stages=d.get("stages_ms"))
p = d.get("parity") or {}
out.update({k: p[k] for k in ("planted_found", "decoys_found", "spot_mismatched_files", "stress_mismatched_files")
            if k in p})
if d.get("cpu_baseline"):
    out["cpu"] = {k: d["cpu_baseline"].get(k) for k in ("value", "files", "files_identical")}
if d.get("full_parity"):
    out["full"] = {k: d["full_parity"][k] for k in ("files", "files_identical", "findings_cpu", "findings_gpu")}
print(json.dumps(out))
EOF
}
for step in "$@"; do
  case "$step" in
    pytest|pytest:*)
      K=()
      [ "$step" != pytest ] && K=(-k "${step#pytest:}")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.log"; exit 1; }
      tail -1 "$O/pytest.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" | cut -c1-240 ;;
    c[0-4]|c[0-4]full)
      N=${step:1:1}
      F=()
      [ "${step#c?}" = full ] && F=(--full-parity)
      timeout -k 10 900 python -u bench.py --config "$N" "${F[@]}" $BENCH_ARGS > "$O/bench_$step.log" 2>&1 \
        || { echo "bench $step failed"; tail -20 "$O/bench_$step.log"; exit 1; }
      echo "$step $(summ "$O/bench_$step.log")" ;;
    trace[0-4])
      N=${step:5:1}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$O/trace_c$N" -o run -- \
        python3 bench.py --config "$N" --steps 5 --warmup 2 --no-cpu --no-parity $BENCH_ARGS \
        > "$O/trace_c$N.log" 2>&1 || { echo "trace $step failed"; tail -20 "$O/trace_c$N.log"; exit 1; }
      echo "$step $(summ "$O/trace_c$N.log")" ;;
    pmc[0-4])
      N=${step:3:1}
      bash tools/pmc.sh "${TAG}_c$N" "$N" || exit 1 ;;
    split)
      timeout -k 10 600 python -u tools/split_bench.py --gb 20 > "$O/split_bench.log" 2>&1 \
        || { echo "split failed"; tail -20 "$O/split_bench.log"; exit 1; }
      tail -5 "$O/split_bench.log" ;;
    exp:*)
      S=${step#exp:}
      TSG_LIB_VARIANT=exp timeout -k 10 900 bash "tools/$S" "$TAG" > "$O/${S%.sh}.log" 2>&1 \
        || { echo "exp $S failed"; tail -20 "$O/${S%.sh}.log"; exit 1; }
      tail -20 "$O/${S%.sh}.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
