# Does the allocation holding an output set its write rate?  K1's store
# pattern over one allocation vs allocations of 2-128 MiB
# (tools/write_probe3.hip), and C5g's PCM images grouped g to an
# allocation (grp<g>) or each at the start of an m-MiB allocation (own<m>)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/write_probe3 > gpurun_out/r06w_probe3.json || { echo "probe failed"; exit 1; }
cat gpurun_out/r06w_probe3.json
L=bjxa_amd/libbjxa.so.0
for lay in sep grp2 grp4 grp8 grp16 grp128 own64 own512 sep; do
timeout -k 10 200 python tools/ab_inproc.py --wl C5g --reps 4 --layout $lay d=$L n64=$L:0x20000 c72=$L:0x20000:140 > gpurun_out/r06w_${lay}.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06w_${lay}.log; exit 1; }
echo "== $lay"; grep -v amdgpu.ids gpurun_out/r06w_${lay}.log
done
