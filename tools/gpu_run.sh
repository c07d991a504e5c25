#!/bin/bash
# One GPU-box session (replaces the per-experiment gpu_r3*.sh launchers):
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]
# Steps, run in order; the first failure ends the session (no GPU work
# after a fault, a time limit or a crash):
#   tests[=<pytest -k expr>]  pytest -m gpu (all, or the selected tests)
#   smoke                     __graft_entry__.smoke()
#   bench[=<args>]            python bench.py <args>, line -> <tag>_bench.json
#   ab=<wl>:<mix>[:<reps>[:<names>]]  tools/ab_inproc.py: this tree's library
#                             against ab/<name>/libbjxa.so.0 for each name of the
#                             comma list (default: every ab/*), interleaved in one
#                             process (ab/ is in .gpurunignore so that the round's
#                             GPU runs do not carry it: drop that line for an A/B
#                             session)
#   abx=<args>                tools/ab_inproc.py <args> as given (layouts, tunings)
#   prof[=<args>]             tools/profile.sh <tag> <args> (trace + counter passes)
#   ktrace=<wl>:<mix>:<names> rocprofv3 --kernel-trace over tools/ab_inproc.py, one
#                             run per library (new = this tree's, else ab/<name>/):
#                             per-kernel median and mean durations of each
#   pmc=<wl>:<mix>:<names>    the same with rocprofv3 --pmc TCC_EA0_RDREQ_sum
#                             TCC_EA0_WRREQ_sum (own pass): bytes per dispatch
# Logs under gpurun_out/<tag>_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
T=$1
shift
mkdir -p gpurun_out
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit 1; }
for step in "$@"; do
	name=${step%%=*}
	arg=
	[ "$name" != "$step" ] && arg=${step#*=}
	case $name in
	tests)
		log=gpurun_out/${T}_gpu.log
		if [ -n "$arg" ]; then
			timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
			    --timeout-method thread -k "$arg" > $log 2>&1 || fail tests $log
		else
			timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
			    --timeout-method thread > $log 2>&1 || fail tests $log
		fi
		tail -1 $log ;;
	smoke)
		log=gpurun_out/${T}_smoke.log
		timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ||
		    fail smoke $log
		tail -1 $log ;;
	bench)
		out=gpurun_out/${T}_bench.json
		# shellcheck disable=SC2086
		timeout -k 10 600 python bench.py $arg > $out 2> gpurun_out/${T}_bench.err ||
		    fail bench gpurun_out/${T}_bench.err
		python3 tools/bench_brief.py $out ;;
	ab)
		IFS=: read -r wl mix reps names <<< "$arg"
		log=gpurun_out/${T}_ab_${wl}_${mix}${names:+_${names//,/_}}.log
		libs="new=bjxa_amd/libbjxa.so.0"
		for d in ab/*/; do
			n=$(basename "$d")
			[ -n "$names" ] && [[ ",$names," != *",$n,"* ]] && continue
			[ -f "$d/libbjxa.so.0" ] && libs="$libs $n=$d/libbjxa.so.0"
		done
		# shellcheck disable=SC2086
		timeout -k 10 600 python tools/ab_inproc.py --wl "$wl" --mix "${mix:-A}" \
		    --reps "${reps:-6}" $libs > $log 2>&1 || fail ab $log
		cat $log ;;
	abx)
		log=gpurun_out/${T}_abx_$(echo "$arg" | tr -c 'A-Za-z0-9' _ | cut -c1-60).log
		# shellcheck disable=SC2086
		timeout -k 10 600 python tools/ab_inproc.py $arg > $log 2>&1 || fail abx $log
		cat $log ;;
	prof)
		# shellcheck disable=SC2086
		bash tools/profile.sh "$T" $arg || exit 1
		python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["kernel_us_alone"], d.get("traffic"))' \
		    gpurun_out/prof_$T/summary.json ;;
	ktrace)
		IFS=: read -r wl mix names <<< "$arg"
		for n in ${names//,/ }; do
			lib=ab/$n/libbjxa.so.0
			[ "$n" = new ] && lib=bjxa_amd/libbjxa.so.0
			d=$PWD/gpurun_out/${T}_kt_${wl}_${mix}_$n
			mkdir -p "$d"
			( export TMPDIR=/tmp; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace \
			    --stats --output-format csv -d "$d" -o run -- python3 \
			    "$OLDPWD/tools/ab_inproc.py" --wl "$wl" --mix "$mix" --reps 3 \
			    "$n=$OLDPWD/$lib" > "$d/log" 2>&1 ) || fail ktrace "$d/log"
			python3 tools/kstats.py "$d/run_kernel_trace.csv" "$n $wl $mix"
		done ;;
	pmc)
		IFS=: read -r wl mix names <<< "$arg"
		for n in ${names//,/ }; do
			lib=ab/$n/libbjxa.so.0
			[ "$n" = new ] && lib=bjxa_amd/libbjxa.so.0
			d=$PWD/gpurun_out/${T}_pmc_${wl}_${mix}_$n
			mkdir -p "$d"
			( export TMPDIR=/tmp; cd /tmp && timeout -s KILL 120 rocprofv3 --pmc \
			    TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d "$d" -o run \
			    -- python3 "$OLDPWD/tools/ab_inproc.py" --wl "$wl" --mix "$mix" \
			    --reps 1 --steps 5 "$n=$OLDPWD/$lib" > "$d/log" 2>&1 ) || fail pmc "$d/log"
			python3 tools/pmc_brief.py "$d" "$n $wl $mix"
		done ;;
	*)
		fail "unknown step $step" ;;
	esac
done
