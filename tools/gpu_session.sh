#!/bin/bash
# tools/gpu_session.sh STEP... -- run GPU steps on the gpurun box, each under
# its own time limit, stopping at the first crash/timeout/abort (never retry).
# Steps: smoke | tests | bench | prof | pmc | residency | power | ... (see case below)
# Steps that pass --ring/--lines/--nt to bench.py run the rejected hot-kernel
# variants: bench.py then loads build_variants/experiments/libbtsha1.so.
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

sampler() {  # sampler FILE N: board power + gfx clock once a second, N times
  for i in $(seq 1 "$2"); do echo "T $(date +%T)"
    timeout 10 amd-smi metric -g 0 -p -c 2>&1 | grep -E "SOCKET_POWER|GFX_0:" -A1; sleep 1; done > "$1" 2>&1
}

rocminfo 2>/dev/null | grep -m1 -E "gfx950" > "$OUT/device.txt" || true
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    tests_new) run pytest_gpu_new 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      -k "multi_device or null_stream or kernel_name or clock_probe or save_chunk" ;;
    pytest:*)
      # a subset of the gpu suite: pytest:<-k expression>
      run "pytest_${step#pytest:}" 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider -k "${step#pytest:}" ;;
    bench) run bench 600 python3 bench.py ;;
    driver_bench)
      # the driver's exact N=1 command (BENCH_rNN.json), timed from outside as well
      t0=$(date +%s%N)
      run driver_bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
      echo "driver_bench outer wall ms: $(( ($(date +%s%N) - t0) / 1000000 ))" | tee -a "$OUT/session.log" ;;
    bench2)
      # two default runs back to back on one box (within-box repeatability of the line)
      run bench_a 600 python3 bench.py && run bench_b 600 python3 bench.py ;;
    bench_rings)
      for r in 2 3 4; do run bench_ring$r 300 python3 bench.py --ring $r --steps 10 --no-cpu-baseline; done ;;
    prof)
      # same process: the bench line (prof.log) and the rocprof kernel stats
      mkdir -p "$OUT/prof"
      run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench \
        -- python3 "$ROOT/bench.py" --steps 20 --no-cpu-baseline --no-host-path --no-clock --power-s 0 ;;
    pmc)
      mkdir -p "$OUT/pmc"
      PB="python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-clock --power-s 0"
      run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o fetch -- $PB
      run pmc_rdreq 600 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc" -o rdreq -- $PB
      run pmc_valu 600 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc" -o valu -- $PB
      run pmc_valu2 600 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES --output-format csv -d "$OUT/pmc" -o valu2 -- $PB
      run pmc_wait 600 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc" -o wait -- $PB ;;
    ubench) run ubench_valu 300 "$ROOT/tools/ubench/valu_rate" ;;
    ubench_alu) run ubench_alu 300 "$ROOT/tools/ubench/sha1_alu" ;;
    mixpattern) run mixpattern 300 "$ROOT/tools/ubench/mixpattern" ;;
    libvariants)
      make -C "$ROOT" -j16 sched_variants > "$OUT/sched_variants_build.log" 2>&1 || exit 2
      for rep in 1 2; do
        for n in default maxilp iterilp maxmem bias0; do
          d="$ROOT/build_variants/$n"
          run "libvar_${n}_$rep" 300 env BT_SHA1_LIB="$d/libbtsha1.so" python3 bench.py --steps 10 --no-cpu-baseline
        done
      done ;;
    dist2)
      # the driver's N>1 launch line, rehearsed with 2 and 4 ranks sharing this box's one GPU
      run dist2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29531 bench.py --gpus 2 --chunks 16384 --steps 5 --warmup 2 --rehearse-shared-gpu
      run dist4 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
        --master-port 29532 bench.py --gpus 4 --chunks 8192 --steps 5 --warmup 2 --rehearse-shared-gpu
      # the driver's other N > 1 shape: no launcher, bench.py starts the ranks itself
      run dist2_self 600 python3 bench.py --gpus 2 --chunks 16384 --steps 5 --warmup 2 --rehearse-shared-gpu ;;
    pairing)
      run pairing 300 "$ROOT/tools/ubench/pairing"
      mkdir -p "$OUT/pairing_pmc"
      run pairing_pmc 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pairing_pmc" -o p -- "$ROOT/tools/ubench/pairing" ;;
    vgprbank) run vgprbank 300 "$ROOT/tools/ubench/vgprbank" ;;
    chain_floor) run chain_floor 300 "$ROOT/tools/ubench/chain_floor" ;;
    order_pmc)
      # co-issue counters per instruction order of the block (compute only)
      mkdir -p "$OUT/order_pmc"
      run order_time 300 "$ROOT/tools/ubench/sha1_order"
      run order_pmc 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE \
        --output-format csv -d "$OUT/order_pmc" -o ord -- "$ROOT/tools/ubench/sha1_order" ;;
    coissue)
      run coissue 300 "$ROOT/tools/ubench/coissue"
      mkdir -p "$OUT/coissue_pmc"
      run coissue_pmc 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/coissue_pmc" -o co -- "$ROOT/tools/ubench/coissue" ;;
    variants)
      for v in "2 1 0" "3 1 0" "4 1 0" "2 2 0" "2 1 1" "3 1 1" "2 2 1"; do
        set -- $v
        run "var_$1$2$3" 300 python3 bench.py --ring $1 --lines $2 --nt $3 --steps 5 --no-cpu-baseline
      done ;;
    pitches)
      for p in 524416 524544 528384 589824; do
        run "pitch_$p" 300 python3 bench.py --pitch $p --steps 5 --no-cpu-baseline
      done ;;
    occupancy)
      run occ_262144 300 python3 bench.py --ring 2 --chunks 262144 --steps 5 --no-cpu-baseline
      run occ_393216 300 python3 bench.py --ring 2 --chunks 393216 --steps 5 --no-cpu-baseline ;;
    occupancy2)
      # round 4: parallelism beyond the workload's 2 waves/SIMD, same box, alternating:
      # one launch of 131072 chunks, one of 262144, two concurrent processes of 131072
      B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-path"
      for rep in 1 2; do
        run "occ_n1_$rep" 200 $B && run "occ_n1_262k_$rep" 200 $B --chunks 262144 && \
        run "occ_n2_$rep" 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
          --master-port 2955$rep bench.py --gpus 2 --steps 20 --warmup 5 --rehearse-shared-gpu || exit 1
      done ;;
    counters) run counters 120 rocprofv3 -L ;;
    residency) run residency 300 "$ROOT/tools/ubench/residency" ;;
    power_residency)
      # ~20 s per mode; power/clock sampled every second alongside
      sampler "$OUT/power_residency_samples.log" 100 &
      sp=$!
      run power_residency 300 "$ROOT/tools/ubench/residency" 131072 1000 1
      echo "T $(date +%T) alu_long start" >> "$OUT/power_residency_samples.log"
      run power_alu_long 300 "$ROOT/tools/ubench/sha1_alu" long 3000
      wait $sp ;;
    power_stream)
      sampler "$OUT/power_stream_samples.log" 60 &
      sp=$!
      run power_stream 300 "$ROOT/tools/ubench/streamread" 400
      wait $sp ;;
    variants597)
      for rep in 1 2; do
        for v in "3 1 0" "2 1 0" "4 1 0" "2 2 0" "10 1 0"; do
          set -- $v
          run "v597_$1$2$3_$rep" 300 python3 bench.py --ring $1 --lines $2 --nt $3 --steps 20 --no-cpu-baseline
        done
      done ;;
    lds_ab)
      for rep in 1 2; do
        run "ab_ring3_$rep" 300 python3 bench.py --ring 3 --steps 20 --no-cpu-baseline
        run "ab_lds_$rep" 300 python3 bench.py --ring 10 --steps 20 --no-cpu-baseline
        run "ab_ldsnt_$rep" 300 python3 bench.py --ring 10 --nt 1 --steps 20 --no-cpu-baseline
      done ;;
    power_valu)
      sampler "$OUT/power_valu_samples.log" 50 &
      sp=$!
      run power_valu 300 "$ROOT/tools/ubench/valu_energy" 4
      wait $sp ;;
    power_lds)
      sampler "$OUT/power_lds_samples.log" 40 &
      sp=$!
      run power_lds 300 python3 bench.py --ring 10 --steps 1500 --warmup 3 --no-cpu-baseline
      wait $sp ;;
    power_stream2)
      sampler "$OUT/power_stream2_samples.log" 90 &
      sp=$!
      run power_stream2 300 "$ROOT/tools/ubench/streamread2" 400
      wait $sp ;;
    wgdist) run wgdist 120 "$ROOT/tools/ubench/wgdist" ;;
    energy_ab)
      # energy per GiB of each hot-kernel variant under the power cap, alternating
      # rounds in one box session (bench.py's `power` object: SMU energy accumulator)
      for rep in 1 2; do
        for v in "3 1 0" "2 1 0" "4 1 0" "2 2 0" "10 1 0" "10 1 1"; do
          set -- $v
          run "energy_$1$2$3_$rep" 300 python3 bench.py --ring $1 --lines $2 --nt $3 --steps 20 \
            --no-cpu-baseline --no-host-path --power-s 4
        done
      done ;;
    power)
      # sample board power and clocks while a ~30 s hot-kernel run is in flight
      ( for i in $(seq 1 12); do date +%T; timeout 10 amd-smi metric -g 0 -p -c 2>&1
          timeout 10 rocm-smi --showpower --showgpuclocks 2>&1; sleep 2; done ) > "$OUT/power_samples.log" 2>&1 &
      sp=$!
      run power_bench 300 python3 bench.py --steps 1500 --warmup 3 --no-cpu-baseline
      wait $sp ;;
    stream)
      python3 -c "import lzma; open('/tmp/C.tar','wb').write(lzma.decompress(open('tests/golden/C.tar.xz','rb').read()))"
      VS="$ROOT/bittorrent-with-congestion-control_amd/bin/verify-stream"
      run stream_pageable 600 python3 tools/stream_bench.py 8
      run vs_packet_b64 300 "$VS" -b 64 -s 2 -r 64 /tmp/C.tar tests/golden/ref_C.chunks
      run vs_packet_b1024 300 "$VS" -b 1024 -s 2 -r 1024 /tmp/C.tar tests/golden/ref_C.chunks
      run vs_zcopy_b1024_s2 300 "$VS" -z -b 1024 -s 2 -r 8 /tmp/C.tar tests/golden/ref_C.chunks
      run vs_zcopy_b2048_s3 300 "$VS" -z -b 2048 -s 3 -r 6 /tmp/C.tar tests/golden/ref_C.chunks
      run vs_zcopy_b256_s4 300 "$VS" -z -b 256 -s 4 -r 32 /tmp/C.tar tests/golden/ref_C.chunks ;;
    stream_z)
      python3 -c "import lzma; open('/tmp/C.tar','wb').write(lzma.decompress(open('tests/golden/C.tar.xz','rb').read()))"
      VS="$ROOT/bittorrent-with-congestion-control_amd/bin/verify-stream"
      run vsz_b2048_s3_p1 300 "$VS" -z -b 2048 -s 3 -r 6 /tmp/C.tar tests/golden/ref_C.chunks
      run vsz_b2048_s3_p256 300 "$VS" -z -b 2048 -s 3 -r 6 -p 256 /tmp/C.tar tests/golden/ref_C.chunks
      run vsz_b1024_s4_p256 300 "$VS" -z -b 1024 -s 4 -r 8 -p 256 /tmp/C.tar tests/golden/ref_C.chunks
      run vsz_b4096_s3_p256 300 "$VS" -z -b 4096 -s 3 -r 4 -p 256 /tmp/C.tar tests/golden/ref_C.chunks ;;
    hostpaths) run stream_pageable 600 python3 tools/stream_bench.py 16 && run stream_pageable8 600 python3 tools/stream_bench.py 8 ;;
    dma_batch)
      for mb in 1024 2048 4096 1024 2048 4096; do
        run "dma_batch_$mb" 300 env BT_SHA1_DMA_BATCH_MB=$mb python3 tools/stream_bench.py 8
      done ;;
    dma_repeat)
      # direct-DMA batch size vs run-to-run rate of the registered path (round 4):
      # call after call in one process, and per NUMA node of the image
      for mb in 4096 1024 2048; do
        run "dr8_$mb" 300 env BT_SHA1_DMA_BATCH_MB=$mb python3 tools/dma_repeat.py 8 5 && \
        run "numa8_$mb" 300 env BT_SHA1_DMA_BATCH_MB=$mb python3 tools/numa_probe.py 8 || exit 1
      done
      run dr32_4096 300 env BT_SHA1_DMA_BATCH_MB=4096 python3 tools/dma_repeat.py 32 4 && \
      run dr32_1024 300 env BT_SHA1_DMA_BATCH_MB=1024 python3 tools/dma_repeat.py 32 4 ;;
    filebench) run filebench 600 env BT_SHA1_TRACE=1 python3 tools/file_bench.py /dev/shm 1 1024 8192 32768 ;;
    filethreads)
      for t in 8 12 16 8 12 16; do
        run "filethreads_$t" 300 env BT_SHA1_TRACE=1 BT_SHA1_COPY_THREADS=$t python3 tools/file_bench.py /dev/shm 8192 32768
      done ;;
    vs_prof)
      python3 -c "import lzma; open('/tmp/C.tar','wb').write(lzma.decompress(open('tests/golden/C.tar.xz','rb').read()))"
      mkdir -p "$OUT/vs_prof"
      run vs_prof 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/vs_prof" -o vs \
        -- "$ROOT/bittorrent-with-congestion-control_amd/bin/verify-stream" -z -b 2048 -s 3 -r 6 /tmp/C.tar tests/golden/ref_C.chunks ;;
    stream_prof)
      mkdir -p "$OUT/stream_prof"
      run stream_prof 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/stream_prof" -o sb \
        -- python3 "$ROOT/tools/stream_bench.py" 4 ;;
    timeline)
      # round 6: kernel + copy trace of 8 GiB pageable chunks_host calls,
      # column-split tail on (default 8 columns) and off; per-call copy span and tail
      for cols in 8 0; do
        mkdir -p "$OUT/tl_$cols"
        run "tl_$cols" 300 env BT_SHA1_COLUMNS=$cols rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
          -d "$OUT/tl_$cols" -o tl -- python3 "$ROOT/tools/pipeline_timeline.py" 4 8 && \
        run "tl_${cols}_summary" 120 python3 tools/pipeline_timeline.py --summary "$OUT/tl_$cols" || exit 1
      done ;;
    latency) run latency 300 python3 tools/latency_bench.py ;;
    numa) run numa 600 python3 tools/numa_probe.py 4 ;;
    copy_order)
      # A/B of the direct-DMA copy order (bt_sha1_api.cpp serial_copies), both legs forced
      for rep in 1 2; do
        run "co_overlap_$rep" 600 env BT_SHA1_COPY_ORDER=overlap python3 tools/numa_probe.py 8 && \
        run "co_serial_$rep" 600 env BT_SHA1_COPY_ORDER=serial python3 tools/numa_probe.py 8 || exit 1
      done ;;
    numa_place)
      # round 6: staging placement (off: left to the kernel; lanes: the lanes'
      # pages on the GPU's node; gpu: lanes + copy threads there) x image node,
      # alternating, median of 5 runs each
      for rep in 1 2; do
        for m in off lanes gpu; do
          run "np_${m}_$rep" 300 env BT_SHA1_NUMA=$m python3 tools/numa_probe.py 8 5 || exit 1
        done
      done ;;
    copythreads)
      for t in 16 12 8 16 12 8; do
        run "ct_$t" 300 env BT_SHA1_COPY_THREADS=$t python3 tools/numa_probe.py 8 5 || exit 1
      done ;;
    pieces)
      for mb in 64 256 128 64 256 128; do
        run "pc_$mb" 300 env BT_SHA1_PIECE_MB=$mb python3 tools/numa_probe.py 8 5 || exit 1
      done ;;
    latency_ab)
      run latency_spin 300 python3 tools/latency_bench.py
      run latency_streamsync 300 env BT_SHA1_SYNC=stream python3 tools/latency_bench.py
      run latency_spin2 300 python3 tools/latency_bench.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done" | tee -a "$OUT/session.log"
