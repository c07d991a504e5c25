#!/bin/bash
# per-wave K1 timeline (XA_DBG_TIMES build): per-XCD end and duration
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
export BJXA_LIB_PATH=tools/bin/ab/times.so.0
timeout -k 10 200 python -u tools/wave_times.py C3 A 0 _m1 > gpurun_out/r3/wt_c3.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/wave_times.py C2 A 0 _m1 > gpurun_out/r3/wt_c2.log 2>&1 || exit $?
python3 - <<'PY'
import json
for f in ("gpurun_out/r3/wt_c3.log", "gpurun_out/r3/wt_c2.log"):
    for l in open(f):
        if l.startswith("{"):
            r = json.loads(l)
            print(f[-10:], round(r["kernel_us"], 1), [round(x) for x in r["per_xcd_end_med"]],
                  [round(x) for x in r["per_xcd_dur_med"]], r["xcd_of_block_mod8"], r["block_mod8_match"])
PY
