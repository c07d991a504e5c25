# C5g's K1 against the PCM images' address bits and the chunk length
# (tools/ab_inproc.py): PCM images in one allocation shifted by
# (37 i mod 64) << b (rot<b>) or spaced 2^b bytes apart (pad<b>), against
# separate allocations; per layout the default plan, 64-eblock chunks
# forced, and 60 / 72 / 76-eblock chunks (batch chunk budgets 116/140/148)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
for lay in sep packed_dst rot8 rot12 rot16 rot20 pad12 pad16 pad20 hipmalloc packed_dst; do
timeout -k 10 200 python tools/ab_inproc.py --wl C5g --reps 4 --layout $lay d=$L n64=$L:0x20000 c60=$L:0x20000:116 c72=$L:0x20000:140 c76=$L:0x20000:148 > gpurun_out/r06v_${lay}.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06v_${lay}.log; exit 1; }
echo "== $lay"; grep -v amdgpu.ids gpurun_out/r06v_${lay}.log
done
