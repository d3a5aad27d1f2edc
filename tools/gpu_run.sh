#!/usr/bin/env bash
# One parameterised GPU-box runner (replaces the per-session tools/gpu_r*.sh one-offs).
#
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh OUT step [step ...]
#
# Every step runs under its own `timeout -k 10`, output goes to gpurun_out/OUT/<step>.*, and
# the first failing step ends the call (set -e: no GPU work after a fault / abort / timeout).
# Steps:
#   smoke            __graft_entry__.smoke()
#   tests            the whole GPU suite (pytest -m gpu, per-test timeout)
#   tests:<expr>     GPU tests selected by -k <expr>
#   files:a,b,..     the GPU tests of tests/test_a_gpu.py, ... in that order (failed asserts do not end the call)
#   envtests:VAR=val the whole GPU suite under one environment setting
#   k20 | k20b       bench.py --steps 20 --warmup 5 (the driver's window), bf16
#   k20f32           the same, --dtype fp32
#   k20f32serial     the same with the fp32 persistent launch off (DNN_PERSIST=0)
#   envk20:VAR=val   k20 with one environment setting
#   abk20:VAR=val[,N] N alternating k20 runs: default env, then VAR=val (same-box A/B)
#   winfit           bench --steps 10..160 with --diag-windows (wall vs event time per window)
#   k20serial | longserial | profserial   the same with the pipelined step off (DNN_PIPELINE=0)
#   k20pipe | longpipe | profpipe         ... and on (DNN_PIPELINE=1)
#   long | long32 | long32serial   bench.py default window (5000 / 500), bf16 / fp32 / fp32 without PERS
#   b2k              bench.py 2000 / 200 steps, no epoch timing (envb2k:VAR=val: under one env setting)
#   profk20          rocprofv3 --kernel-trace over the driver's 20/5 window (+3 diagnostic windows)
#   prof | prof32    rocprofv3 --kernel-trace --stats over 2000 steps (bf16 / fp32)
#   pmc:<c1,c2,..>   one rocprofv3 --pmc pass over 200 bf16 steps (counters comma-separated)
#   pmcserial:<..>   the same with the pipelined step off
#   hostprobe[:VAR=val]  host-side cost of the timed window (launch paths, sync styles)
#   floor[:A=1+B=2]  launch + synchronize floor and the 20-step window under runtime settings
#   aqlwin[:steps]   graph replay vs direct AQL dispatch of the persistent window (timing + bits)
#   phase | phase32 | phase32pers | phasepipe | phasepers  per-phase timeline of the fused kernels (tools/phase_trace*.py; pipelined launch)
#   rehearse2        2 ranks on this GPU, no torchrun: DNN_BACKEND=gloo bench.py --gpus 2 (self-launch + A/B)
#   fault2 | fault4  tools/fault_bench.py -n 2|4 --share-gpu (rank-drop recovery latency)
#   sweep:<b1,b2,..> bench.py --batch-size b for each b (2000 / 200 steps)
#   racehunt:N[:variants[:VAR=val[:extra args]]]  tools/race_hunt.py (long run under load vs serial, per variant)
#   abso:NAME[,N]    N alternating k20 runs: main build, then ops/variants/NAME.so (kernel A/B)
#   useso:NAME       use distributed_neural_network_amd/ops/variants/NAME.so from here on (kernel A/B;
#                    the original extension is restored when the script exits)
#   inproc[:args]    tools/inproc_pair.py (2 in-process ranks on this GPU: exchange forms, JSON)
#   inproctrace:f,.. tools/inproc_pair.py --trace (per-block waits, per-step starts of those forms)
#   diverge[:a,b]   tools/inproc_diverge.py (when the in-process ranks' replicas part; args comma-separated)
#   streamprobe[:a,b] tools/inproc_stream_probe.py (does the harness depend on streams created before it?)
#   export:VAR=val   export for the later steps (their output names get _VAR)
#   inject2[:VAR=val]   2 self-launched ranks on this GPU, rank 1 killed in the xGMI set-up of launch
#                    attempt 1 (DNN_INJECT_XGMI_SETUP_FAIL=1): the launcher's retry in fresh ranks
#   torchrun2[:VAR=val] 2 ranks under torchrun (per-rank supervisors); torchrun2inject: + the injection
#   vgg              layer engine, cifar-vgg bf16 / fp32, split-K fc1 forward on / off
set -e
O=gpurun_out/${1:?usage: gpu_run.sh OUT step...}
SO=distributed_neural_network_amd/ops/_dnn_hip.cpython-310-x86_64-linux-gnu.so
restore_so() { [ -f "$SO.orig" ] && mv -f "$SO.orig" "$SO"; return 0; }
trap restore_so EXIT
shift
mkdir -p "$O"
export TMPDIR=/tmp
USESO=""  # "_NAME" after useso:NAME (suffix of the later steps' output names)
stamp() { echo "[gpu_run $(date +%H:%M:%S)] $*"; }
for s in "$@"; do
  stamp "step $s"
  case "$s" in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    tests) timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
             > "$O/tests.log" 2>&1 ;;
    envtests:*)  # the whole GPU suite under one env setting: envtests:VAR=value
      kv="${s#envtests:}"; n=$(echo "$kv" | tr '=/' '__')
      env "$kv" timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
             > "$O/tests_$n.log" 2>&1 ;;
    tests:*) timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
             -k "${s#tests:}" > "$O/tests_k.log" 2>&1 ;;
    export:*)  # export:VAR=val for the later steps of this call (their output names get _VAR)
      kv="${s#export:}"; export "${kv?}"; USESO="${USESO}_${kv%%=*}" ;;
    files:*)  # files:a,b,...: the GPU tests of tests/test_<a>_gpu.py, ... in that order (one process)
      fs=""; for f in $(echo "${s#files:}" | tr ',' ' '); do fs="$fs tests/test_${f}_gpu.py"; done
      n=$(echo "${s#files:}" | tr ',' '_')
      # (exit 1 = failed assertions only: the call goes on; a crash, abort or time limit ends it)
      rc=0; timeout -k 10 900 python -u -m pytest $fs -m gpu -v --timeout 300 --timeout-method thread \
             > "$O/files_$n$USESO.log" 2>&1 || rc=$?
      [ "$rc" -le 1 ] || exit "$rc" ;;
    k20|k20b) timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/$s.json" 2> "$O/$s.err" ;;
    k20pipe) DNN_PIPELINE=1 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/$s.json" 2> "$O/$s.err" ;;
    longpipe) DNN_PIPELINE=1 timeout -k 10 300 python bench.py > "$O/$s.json" 2> "$O/$s.err" ;;
    k20serial) DNN_PIPELINE=0 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/$s.json" 2> "$O/$s.err" ;;
    longserial) DNN_PIPELINE=0 timeout -k 10 300 python bench.py > "$O/$s.json" 2> "$O/$s.err" ;;
    envk20:*)  # the driver's window under one runtime env setting: envk20:VAR=value
      kv="${s#envk20:}"; n=$(echo "$kv" | tr '=/' '__')
      env "$kv" timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/k20_$n.json" 2> "$O/k20_$n.err" ;;
    abk20:*)  # abk20:VAR=val[,N]: N alternating driver windows (default env, then VAR=val) - a same-box A/B
      spec="${s#abk20:}"; kv="${spec%%,*}"; n=3; [ "$spec" != "$kv" ] && n="${spec#*,}"
      nm=$(echo "$kv" | tr '=/' '__')
      for i in $(seq 1 "$n"); do
        timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/abk20_${nm}_${i}_base.json" 2> "$O/abk20_${nm}_${i}_base.err"
        env "$kv" timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/abk20_${nm}_${i}_var.json" \
          2> "$O/abk20_${nm}_${i}_var.err"
      done ;;
    winfit|winfit:*)  # the window's fixed cost: bench at several step counts, wall vs GPU events per
      # window (winfit:VAR=val[,k1,k2..]: under one env setting, for the given step counts)
      spec="${s#winfit}"; spec="${spec#:}"; kv="${spec%%,*}"; ks="10 20 40 80 160"
      [ "$spec" != "$kv" ] && ks=$(echo "${spec#*,}" | tr ',' ' ')
      [ -z "$kv" ] && kv="DNN_NOTHING=0"; n=$(echo "$kv" | tr '=/' '__')
      for k in $ks; do
        env "$kv" timeout -k 10 150 python bench.py --steps $k --warmup 5 --diag-windows 3 \
          > "$O/winfit_${n}_k$k.json" 2> "$O/winfit_${n}_k$k.err"
      done ;;
    k20f32) timeout -k 10 150 python bench.py --dtype fp32 --steps 20 --warmup 5 > "$O/$s.json" 2> "$O/$s.err" ;;
    k20f32serial) DNN_PERSIST=0 timeout -k 10 150 python bench.py --dtype fp32 --steps 20 --warmup 5 > "$O/$s.json" \
                    2> "$O/$s.err" ;;
    long) timeout -k 10 300 python bench.py > "$O/long.json" 2> "$O/long.err" ;;
    b2k) timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-epoch > "$O/b2k.json" 2> "$O/b2k.err" ;;
    envb2k:*)  # b2k under one runtime env setting: envb2k:VAR=value
      kv="${s#envb2k:}"; n=$(echo "$kv" | tr '=/' '__')
      env "$kv" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-epoch > "$O/b2k_$n.json" 2> "$O/b2k_$n.err" ;;
    envphasepers:*)  # phasepers under one runtime env setting
      kv="${s#envphasepers:}"; n=$(echo "$kv" | tr '=/' '__')
      env "$kv" timeout -k 10 300 python tools/phase_trace.py --pers > "$O/phasepers_$n.txt" 2>&1 ;;
    long32) timeout -k 10 300 python bench.py --dtype fp32 > "$O/long32.json" 2> "$O/long32.err" ;;
    long32serial) DNN_PERSIST=0 timeout -k 10 300 python bench.py --dtype fp32 > "$O/$s.json" 2> "$O/$s.err" ;;
    long32pers) DNN_PERSIST_F32=1 timeout -k 10 300 python bench.py --dtype fp32 > "$O/$s.json" 2> "$O/$s.err" ;;
    k20f32pers) DNN_PERSIST_F32=1 timeout -k 10 150 python bench.py --dtype fp32 --steps 20 --warmup 5 > "$O/$s.json" \
                  2> "$O/$s.err" ;;
    prof|prof32|profserial|profpipe)
      dt=bf16; [ "$s" = prof32 ] && dt=fp32
      [ "$s" = profserial ] && export DNN_PIPELINE=0
      [ "$s" = profpipe ] && export DNN_PIPELINE=1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d "$O/$s" -o run -- \
        python3 bench.py --dtype $dt --steps 2000 --warmup 200 --no-epoch > "$O/$s.log" 2>&1
      db=$(find "$O/$s" -name '*.db' | head -n 1 || true)
      [ -n "$db" ] && python tools/kstats.py "$db" --steps 2200 > "$O/${s}_kernel_stats.txt" 2>&1 || true
      unset DNN_PIPELINE ;;
    profk20)  # kernel trace of the driver's window (kernel span vs the bench's wall time per window)
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$s" -o run -- \
        python3 bench.py --steps 20 --warmup 5 --diag-windows 3 > "$O/$s.log" 2>&1 ;;
    pmc:*|pmcserial:*)
      c="${s#*:}"; n=$(echo "$c" | tr ',' '_' | cut -c1-60); pre=pmc
      [ "${s%%:*}" = pmcserial ] && { export DNN_PIPELINE=0; pre=pmcserial; }
      timeout -s KILL 90 rocprofv3 --pmc ${c//,/ } --kernel-trace --output-format csv -d "$O/${pre}_$n" -o run -- \
        python3 bench.py --steps 200 --warmup 20 --no-epoch > "$O/${pre}_$n.log" 2>&1
      unset DNN_PIPELINE ;;
    phase) timeout -k 10 300 python tools/phase_trace.py > "$O/phase.txt" 2>&1 ;;
    phasepipe) timeout -k 10 300 python tools/phase_trace.py --pipe > "$O/phasepipe.txt" 2>&1 ;;
    phasepers) timeout -k 10 300 python tools/phase_trace.py --pers > "$O/phasepers.txt" 2>&1 ;;
    hostprobe|hostprobe:*)  # host-side cost of the timed window (tools/window_host_probe.py); hostprobe:VAR=val
      kv="${s#hostprobe}"; kv="${kv#:}"; [ -z "$kv" ] && kv="DNN_NOTHING=0"; n=$(echo "$kv" | tr '=/' '__')
      env "$kv" timeout -k 10 200 python tools/window_host_probe.py > "$O/hostprobe_$n.json" 2> "$O/hostprobe_$n.err" ;;
    floor|floor:*)  # tools/launch_floor_probe.py under runtime settings floor:A=1+B=2 (launch + sync floor)
      kv="${s#floor}"; kv="${kv#:}"; [ -z "$kv" ] && kv="DNN_NOTHING=0"; n=$(echo "$kv" | tr '=/+' '___')
      env $(echo "$kv" | tr '+' ' ') timeout -k 10 120 python tools/launch_floor_probe.py > "$O/floor_$n.json" \
        2> "$O/floor_$n.err" ;;
    aqlwin|aqlwin:*)  # tools/aql_window.py: graph replay vs direct AQL dispatch windows + bits (aqlwin:FENCE)
      f="${s#aqlwin}"; f="${f#:}"; [ -z "$f" ] && f=ss
      DNN_AQL_FENCE=$f timeout -k 10 120 python tools/aql_window.py 20 > "$O/aqlwin_$f.json" 2> "$O/aqlwin_$f.err" ;;
    pipeflags:*)  # the pipelined step's variants: phase trace + 2000-step bench per DNN_PIPE_FLAGS value
      for f in $(echo "${s#pipeflags:}" | tr ',' ' '); do
        DNN_PIPE_FLAGS=$f timeout -k 10 300 python tools/phase_trace.py --pipe > "$O/phasepipe_f$f.txt" 2>&1
        DNN_PIPE_FLAGS=$f DNN_PIPELINE=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-epoch \
          > "$O/b2k_pipe_f$f.json" 2> "$O/b2k_pipe_f$f.err"
      done
      DNN_PIPELINE=0 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-epoch > "$O/b2k_serial.json" \
        2> "$O/b2k_serial.err" ;;
    b2kenv:*)  # phase trace + 2000-step bench of the pipelined step under one env setting (VAR=val)
      kv="${s#b2kenv:}"; n=$(echo "$kv" | tr '=/' '__')
      env "$kv" timeout -k 10 300 python tools/phase_trace.py --pipe > "$O/phasepipe_$n.txt" 2>&1
      env "$kv" DNN_PIPELINE=1 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-epoch \
        > "$O/b2k_$n.json" 2> "$O/b2k_$n.err" ;;
    phase32) timeout -k 10 300 python tools/phase_trace_f32.py > "$O/phase32.txt" 2>&1 ;;
    phase32pers) timeout -k 10 300 python tools/phase_trace_f32.py --pers > "$O/phase32pers.txt" 2>&1 ;;
    rehearse2) DNN_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 \
                 > "$O/rehearse2.json" 2> "$O/rehearse2.err" ;;
    rehearse2diag) DNN_BACKEND=gloo DNN_AB_DEBUG=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 \
                 --diag-windows 3 > "$O/$s.json" 2> "$O/$s.err" ;;
    fault2) timeout -k 10 400 python tools/fault_bench.py -n 2 --share-gpu > "$O/fault2.json" 2> "$O/fault2.log" ;;
    fault4) timeout -k 10 400 python tools/fault_bench.py -n 4 --share-gpu > "$O/fault4.json" 2> "$O/fault4.log" ;;
    vgg) for dt in bf16 fp32; do for sk in 1 0; do
           DNN_LINEAR_SPLITK=$sk timeout -k 10 200 python bench.py --model cifar-vgg --dtype $dt --steps 300 --warmup 30 \
             --no-epoch > "$O/vgg_${dt}_splitk$sk.json" 2> "$O/vgg_${dt}_splitk$sk.err"
         done; done ;;
    sweep:*)
      for b in $(echo "${s#sweep:}" | tr ',' ' '); do
        timeout -k 10 200 python bench.py --batch-size "$b" --steps 2000 --warmup 200 --no-epoch \
          > "$O/sweep_b$b.json" 2> "$O/sweep_b$b.err"
      done ;;
    racehunt:*)  # racehunt:N[:variants[:VAR=val]] tools/race_hunt.py: the long-run-under-load comparison per variant
      IFS=: read -r _ n vs kv xa <<< "$s"; [ -z "$vs" ] && vs=bf16-pipe,bf16-pers,fp32-pers; [ -z "$kv" ] && kv="DNN_NOTHING=0"
      tag=$(echo "${vs}_${kv}_$xa" | tr ',=/ ' '-___')
      env "$kv" timeout -k 10 500 python tools/race_hunt.py --rounds "$n" --variants "$vs" $xa > "$O/racehunt_$tag.txt" 2>&1 ;;
    useso:*)  # A/B of kernel builds in one call: copy ops/variants/NAME.so over the live extension
      [ -f "$SO.orig" ] || cp "$SO" "$SO.orig"
      cp "distributed_neural_network_amd/ops/variants/${s#useso:}.so" "$SO"
      USESO="_${s#useso:}" ;;
    abso:*)  # abso:NAME[,N]: N alternating k20 runs, main build then ops/variants/NAME.so (kernel A/B)
      spec="${s#abso:}"; nm="${spec%%,*}"; n=3; [ "$spec" != "$nm" ] && n="${spec#*,}"
      [ -f "$SO.orig" ] || cp "$SO" "$SO.orig"
      for i in $(seq 1 "$n"); do
        cp "$SO.orig" "$SO"
        timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/abso_${nm}_${i}_base.json" 2> "$O/abso_${nm}_${i}_base.err"
        cp "distributed_neural_network_amd/ops/variants/$nm.so" "$SO"
        timeout -k 10 150 python bench.py --steps 20 --warmup 5 > "$O/abso_${nm}_${i}_var.json" 2> "$O/abso_${nm}_${i}_var.err"
      done
      cp "$SO.orig" "$SO" ;;
    inproctrace:*)
      f="${s#inproctrace:}"; n=$(echo "$f" | tr ',' '_')$USESO
      timeout -k 10 300 python tools/inproc_pair.py --trace "$f" > "$O/inproctrace_$n.json" 2> "$O/inproctrace_$n.err" ;;
    inproc|inproc:*)
      xa="${s#inproc}"; xa="${xa#:}"; n=$(echo "inproc_$xa" | tr ' =/-' '____')$USESO
      timeout -k 10 400 python tools/inproc_pair.py $xa > "$O/$n.json" 2> "$O/$n.err" ;;
    diverge|diverge:*)  # tools/inproc_diverge.py [args, spaces as commas]: when do the in-process ranks part?
      xa=$(echo "${s#diverge}" | sed 's/^://; s/,/ /g'); n=$(echo "dv_$xa" | tr ' =/-' '____')$USESO
      timeout -k 10 500 python tools/inproc_diverge.py $xa > "$O/$n.json" 2> "$O/$n.err" ;;
    streamprobe|streamprobe:*)  # tools/inproc_stream_probe.py [args, spaces as commas]
      xa=$(echo "${s#streamprobe}" | sed 's/^://; s/,/ /g'); n=$(echo "sp_$xa" | tr ' =/-' '____')$USESO
      timeout -k 10 600 python tools/inproc_stream_probe.py $xa > "$O/$n.json" 2> "$O/$n.err" ;;
    inject2|inject2:*)
      kv="${s#inject2}"; kv="${kv#:}"; [ -z "$kv" ] && kv="DNN_NOTHING=0"; n=$(echo "$kv" | tr '=/' '__')
      env "$kv" DNN_INJECT_XGMI_SETUP_FAIL=1 DNN_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 20 \
        --warmup 5 > "$O/inject2_$n.json" 2> "$O/inject2_$n.err" ;;
    torchrun2|torchrun2:*|torchrun2inject)
      kv="${s#torchrun2}"; kv="${kv#:}"; [ -z "$kv" ] && kv="DNN_NOTHING=0"
      [ "$s" = torchrun2inject ] && kv="DNN_INJECT_XGMI_SETUP_FAIL=1"
      n=$(echo "$kv" | tr '=/' '__')
      env "$kv" DNN_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
        > "$O/torchrun2_$n.json" 2> "$O/torchrun2_$n.err" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  stamp "done $s"
done
