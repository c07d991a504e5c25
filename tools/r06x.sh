# C5g's PCM images in physically contiguous memory (hipDeviceMallocContiguous):
# packed in one such allocation, or one each; against torch's separate
# tensors and one plain allocation (packed_dst)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
L=bjxa_amd/libbjxa.so.0
for lay in sep contig packed_dst contig_sep grp3 contig sep; do
timeout -k 10 200 python tools/ab_inproc.py --wl C5g --reps 4 --layout $lay d=$L n64=$L:0x20000 > gpurun_out/r06x_${lay}.log 2>&1 || { echo "ab failed $lay"; tail gpurun_out/r06x_${lay}.log; exit 1; }
echo "== $lay"; grep -v amdgpu.ids gpurun_out/r06x_${lay}.log
done
