#!/bin/bash
# One parameterised GPU-box cycle (replaces the per-cycle gpu_r3*.sh scripts of round 3).
#   bash tools/cycle.sh TAG STEPS [bench args...]
# STEPS: comma-separated, run in order, stopping at the first failure:
#   tests         every -m gpu test           tests:<pytest args>  e.g. tests:tests/test_gpu_parity.py
#   smoke         __graft_entry__.smoke()
#   bench         the default bench line (bench args appended) -> bench.json
#   kt            rocprofv3 kernel trace + stats of a short k26w bench run
#   calib         FETCH_SIZE calibration: tools/calib/pj_gather_calib timed, then under --pmc (one counter
#                 group per run) -> calib.log, calpmc_*/, gather_calib.json (tools/calib_table.py)
#   wtable        the per-kernel table of k26w solves: kernel trace + --pmc passes (RDREQ / RDREQ_32B,
#                 FETCH_SIZE, WRITE_SIZE) of tools/traffic_probe.py, its work counters -> pmc_table.txt,
#                 traffic_k26w.json (tools/pmc_solve_table.py, calibrated by gather_calib.json: this
#                 cycle's calib step if it ran, else profiles/r06/gather_calib.json)
#   klevels[:opts] per-level table of configs[1] (K22 BFS): tools/k22_levels.py under a kernel trace and --pmc
#                 passes -> k22_levels.txt (tools/k22_level_table.py); opts = libpj options k=v~k=v
#   probe:<cmd>   any python command line under a 240 s limit (e.g. probe:tools/probe_ms.py)
#   vtests:<v>:<pytest args>  -m gpu tests under the libpj build variant <v>
#   ktp:<cmd>     rocprofv3 kernel trace + stats of any python command line -> kt_<name>/
#   vktp:<v>:<cmd>  the same under the libpj build variant <v> -> kt_<v>_<name>/
#   abp:<v1+v2..>:<python args>  interleaved A/B (ABP_PASSES times, default AB_PASSES) of any probe under
#                 build variants -> abp_<v>.<pass>.log
#   abo:<o1+o2..> interleaved A/B of the k26w bench line under libpj option sets (o = k=v/k=v...,
#                 "default" = none), AB_PASSES times
#   ab:<v1+v2..>  interleaved A/B (AB_PASSES times, default 2) of the k26w bench line under libpj
#                 build variants (lib/variants/<v>/libpj.so; "default" = the main build)
# Inside a step's arguments "~" stands for a space and "^" for a comma (STEPS is one word).
# Output under gpurun_out/TAG.
set -o pipefail
TAG=${1:?tag}; STEPS=${2:?steps}; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
IFS=',' read -ra LIST <<< "$STEPS"
for st in "${LIST[@]}"; do
  name=${st%%:*}; arg=""; [[ "$st" == *:* ]] && arg=${st#*:}
  arg=${arg//\~/ }; arg=${arg//^/,}
  echo "== $name $arg"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${arg:-tests} \
        > "$OUT/pytest_gpu.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
      tail -1 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 500 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d.get('secondary',{}); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('time_to_solution_s'), (d.get('time_to_solution_phases') or {}).get('process_phases'), s.get('wg',{}).get('ms_per_sssp'), s.get('ms1024',{}).get('batch_ms'))" "$OUT/bench.json" ;;
    kt)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
        python3 bench.py --no-cpu-baseline --no-secondary --no-partitioned --no-tts --steps 8 --warmup 1 "$@" \
        > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail "$OUT/kt.log"; exit 1; } ;;
    calib)
      B=tools/calib/pj_gather_calib
      timeout -k 10 120 $B 4096 3 > "$OUT/calib.log" 2>&1 || { echo "calib failed"; tail "$OUT/calib.log"; exit 1; }
      for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum" FETCH_SIZE WRITE_SIZE; do
        gn=$(echo "$grp" | tr ' ' '+')
        timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/calpmc_$gn" -o run -- $B 4096 3 \
          > "$OUT/calpmc_$gn.log" 2>&1 || { echo "calib pmc $grp failed"; tail "$OUT/calpmc_$gn.log"; exit 1; }
      done
      python3 tools/calib_table.py "$OUT" > "$OUT/gather_calib.json" || { echo "calib table failed"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bytes/request', d.get('bytes_per_request'), 'dword gathers/s', d.get('random_dword_gathers_per_s'))" "$OUT/gather_calib.json" ;;
    wtable)
      P="tools/traffic_probe.py 26 ${WT_SOLVES:-6} 1"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wkt" -o run -- python3 -u $P \
        --json "$OUT/probe_work.json" > "$OUT/wkt.log" 2>&1 || { echo "wtable trace failed"; tail "$OUT/wkt.log"; exit 1; }
      for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" FETCH_SIZE WRITE_SIZE; do
        gn=$(echo "$grp" | tr ' ' '+')
        timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d "$OUT/wpmc_$gn" -o run -- python3 -u $P \
          > "$OUT/wpmc_$gn.log" 2>&1 || { echo "wtable pmc $grp failed"; tail "$OUT/wpmc_$gn.log"; exit 1; }
      done
      CAL=profiles/r06/gather_calib.json; [ -f "$OUT/gather_calib.json" ] && CAL="$OUT/gather_calib.json"
      python3 tools/pmc_solve_table.py "$OUT" "$CAL" > "$OUT/pmc_table.txt" 2>&1 || { echo "table failed"; cat "$OUT/pmc_table.txt"; exit 1; }
      cat "$OUT/pmc_table.txt" ;;
    klevels)
      P="tools/k22_levels.py ${KL_ROOTS:-4} $arg"
      KT=$(echo "$arg" | tr -c 'A-Za-z0-9_\n' '_'); KO="$OUT/kl${KT:+_$KT}"; mkdir -p "$KO"
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$KO/klkt" -o run -- python3 -u $P \
        > "$KO/klkt.log" 2> "$KO/klevels.log" || { echo "klevels trace failed"; tail "$KO/klevels.log"; exit 1; }
      for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" FETCH_SIZE WRITE_SIZE; do
        gn=$(echo "$grp" | tr ' ' '+')
        timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$KO/klpmc_$gn" -o run -- python3 -u $P \
          > "$KO/klpmc_$gn.log" 2>&1 || { echo "klevels pmc $grp failed"; tail "$KO/klpmc_$gn.log"; exit 1; }
      done
      CAL=profiles/r06/gather_calib.json; [ -f "$OUT/gather_calib.json" ] && CAL="$OUT/gather_calib.json"
      python3 tools/k22_level_table.py "$KO" "$CAL" > "$KO/k22_levels.txt" 2>&1 || { echo "level table failed"; cat "$KO/k22_levels.txt"; exit 1; }
      tail -8 "$KO/k22_levels.txt" ;;
    probe)
      PN=$((PN + 1))  # (a step number: repeated probes of one command keep their logs)
      timeout -k 10 240 python3 -u $arg > "$OUT/probe_$(echo "$arg" | tr -c 'A-Za-z0-9' '_' | cut -c1-24)_$(echo "$arg" | md5sum | cut -c1-6)_$PN.log" 2>&1 \
        || { echo "probe failed: $arg"; exit 1; } ;;
    vtests)
      v=${arg%%:*}; targs=${arg#*:}
      PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so timeout -k 10 600 python -u -m pytest -x -q \
        --timeout 300 --timeout-method thread -m gpu $targs > "$OUT/vtests_$v.log" 2>&1 \
        || { echo "vtests $v failed"; tail -30 "$OUT/vtests_$v.log"; exit 1; }
      tail -1 "$OUT/vtests_$v.log" ;;
    ktp)
      kn=kt_$(echo "$arg" | tr -c 'A-Za-z0-9' '_' | cut -c1-30)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$kn" -o run -- python3 -u $arg \
        > "$OUT/$kn.log" 2>&1 || { echo "ktp failed: $arg"; tail "$OUT/$kn.log"; exit 1; } ;;
    vktp)
      v=${arg%%:*}; cmd=${arg#*:}; kn=kt_${v}_$(echo "$cmd" | tr -c 'A-Za-z0-9' '_' | cut -c1-30)
      PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so timeout -k 10 300 rocprofv3 --kernel-trace \
        --stats --output-format csv -d "$OUT/$kn" -o run -- python3 -u $cmd > "$OUT/$kn.log" 2>&1 \
        || { echo "vktp failed: $arg"; tail "$OUT/$kn.log"; exit 1; } ;;
    abp)
      vl=${arg%%:*}; cmd=${arg#*:}
      IFS='+' read -ra VS <<< "$vl"
      for pass in $(seq 1 ${ABP_PASSES:-${AB_PASSES:-2}}); do
        for v in "${VS[@]}"; do
          if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
          timeout -k 10 240 python3 -u $cmd > "$OUT/abp_$v.$pass.log" 2>&1 || { echo "abp $v failed"; tail -5 "$OUT/abp_$v.$pass.log"; exit 1; }
          echo "== $v $pass"; grep -v "^Warn\|amdgpu.ids" "$OUT/abp_$v.$pass.log" | tail -4
        done
      done
      unset PJ_LIB_OVERRIDE ;;
    abo)
      IFS='+' read -ra OS <<< "$arg"
      for pass in $(seq 1 ${AB_PASSES:-2}); do
        for o in "${OS[@]}"; do
          optargs=""; IFS='/' read -ra KV <<< "$o"
          for kv in "${KV[@]}"; do [ "$kv" != default ] && optargs="$optargs --opt $kv"; done
          tag=$(echo "$o" | tr -c 'A-Za-z0-9' '_')
          timeout -k 10 200 python3 -u bench.py --no-secondary --no-partitioned --no-tts --no-cpu-baseline --steps 32 --warmup 4 $optargs "$@" \
            > "$OUT/abo_$tag.$pass.json" 2> "$OUT/abo_$tag.$pass.err" || { echo "abo $o failed"; tail -5 "$OUT/abo_$tag.$pass.err"; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['frac'])" "$OUT/abo_$tag.$pass.json" "$o" $pass
        done
      done ;;
    ab)
      IFS='+' read -ra VS <<< "$arg"
      for pass in $(seq 1 ${AB_PASSES:-2}); do
        for v in "${VS[@]}"; do
          if [ "$v" != default ]; then export PJ_LIB_OVERRIDE=$PWD/paralleljohnson_amd/lib/variants/$v/libpj.so; else unset PJ_LIB_OVERRIDE; fi
          timeout -k 10 200 python3 -u bench.py --no-secondary --no-partitioned --no-tts --no-cpu-baseline --steps 32 --warmup 4 "$@" \
            > "$OUT/ab_$v.$pass.json" 2> "$OUT/ab_$v.$pass.err" || { echo "ab $v failed"; tail -5 "$OUT/ab_$v.$pass.err"; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['frac'])" "$OUT/ab_$v.$pass.json" $v $pass
        done
      done
      unset PJ_LIB_OVERRIDE ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "cycle ok"
