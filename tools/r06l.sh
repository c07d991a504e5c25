# C5g's K1 in the torch layout of tools/ab_inproc.py, four fresh processes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
for i in 1 2 3 4; do
for lay in sep hipmalloc; do
timeout -k 10 300 python tools/ab_inproc.py --wl C5g --reps 4 --layout $lay new=$L > gpurun_out/r06l_${lay}_$i.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06l_${lay}_$i.log; exit 1; }
echo "$lay $i $(grep -v amdgpu.ids gpurun_out/r06l_${lay}_$i.log)"
done
done
