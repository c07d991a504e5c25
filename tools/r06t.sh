# C5g's K1 across buffer layouts, every layout in fresh processes, the
# layouts interleaved (tools/ab_inproc.py; round-6 re-check of R6-5's
# packed case, which had been measured only in a box's first processes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
for i in 1 2 3; do
for lay in sep packed hipmalloc packed_src packed_dst pages; do
timeout -k 10 200 python tools/ab_inproc.py --wl C5g --reps 4 --layout $lay new=$L > gpurun_out/r06t_${lay}_$i.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06t_${lay}_$i.log; exit 1; }
echo "$lay $i $(grep -v amdgpu.ids gpurun_out/r06t_${lay}_$i.log)"
done
done
