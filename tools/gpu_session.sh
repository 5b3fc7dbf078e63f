#!/bin/bash
# tools/gpu_session.sh STEP... -- run GPU steps on the gpurun box, each under
# its own time limit, stopping at the first crash/timeout/abort (never retry).
# Steps: smoke | tests | bench | prof | pmc | scale
# Outputs land in gpurun_out/ (merged back by gpurun).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0

run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] >>> $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] <<< $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 25 "$OUT/$name.log"
  case $rc in
    0|1|5) return 0 ;;        # ok / test failures / no tests: safe to go on
    *) echo "STOP: $name exited $rc" | tee -a "$OUT/session.log"; exit $rc ;;
  esac
}

rocminfo 2>/dev/null | grep -m1 -E "gfx950" > "$OUT/device.txt" || true
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    bench) run bench 600 python3 bench.py ;;
    bench_rings)
      for r in 2 3 4; do run bench_ring$r 300 python3 bench.py --ring $r --steps 10 --no-cpu-baseline; done ;;
    prof)
      mkdir -p "$OUT/prof"
      run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench \
        -- python3 "$ROOT/bench.py" --steps 10 --no-cpu-baseline ;;
    pmc)
      mkdir -p "$OUT/pmc"
      run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o fetch \
        -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
      run pmc_rdreq 600 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$OUT/pmc" -o rdreq \
        -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
      run pmc_valu 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc" -o valu \
        -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done" | tee -a "$OUT/session.log"
