/*
 * xa_files.hip -- many host streams in one batched GPU pass
 * (bjxa_hip_decode_files -> bjxa__gpu_decode_many).
 *
 * Host side of the file-level batch: the callers'
 * XA block data is gathered into the device input image and the decoded PCM
 * scattered back out.  Measured: 1024 separate PCIe copies
 * into the callers' own buffers ran at 24-29 GB/s, against ~56 GB/s for one
 * large copy from pinned memory.  So the images move in large slabs through
 * two pinned staging buffers, and a small pool of host threads copies
 * between the staging slabs and the callers' buffers:
 *
 *   in:   gather slab k (threads)  ||  H2D slab k-1   (two buffers)
 *   out:  D2H slab k+1             ||  scatter slab k (threads)
 *
 * The staging buffers, device images and threads persist across calls
 * (one process-wide context behind a mutex); nothing keeps a pointer to a
 * caller's buffer after the call returns.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "xa_decode.h"
#include "xa_pool.h"
#include "xa_gpu.h"
#include "../../include/bjxa_hip.h"

#ifdef XA_FILES_TIMING
#include <stdio.h>
#include <time.h>
static double
now_ms(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}
#define TMARK(name) do { (void)hipStreamSynchronize(c.stream); \
	fprintf(stderr, "%s %.2f\n", name, now_ms() - t0); } while (0)
#else
#define TMARK(name) do { } while (0)
#endif

namespace {

using xa_pool::piece;
using xa_pool::copy_pool;
using xa_pool::pool_threads;

/* slab size of the pinned staging buffers */
constexpr size_t SLAB = (size_t)64 << 20;

struct files_ctx {
	std::mutex m;
	bool ready = false;
	hipStream_t stream = NULL;
	hipEvent_t ev[2] = { NULL, NULL };
	uint8_t *h_slab[2] = { NULL, NULL };	/* pinned */
	uint8_t *d_in = NULL, *d_out = NULL;
	uint32_t *d_st = NULL;
	size_t in_cap = 0, out_cap = 0, st_cap = 0;
	void *d_bws = NULL;			/* batch workspace, kept */
	size_t bws_cap = 0;
	copy_pool *pool = NULL;
};

files_ctx ctx;

int
setup(files_ctx &c)
{
	if (c.ready)
		return 0;
	if (hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) !=
	    hipSuccess)
		return -1;
	for (int i = 0; i < 2; i++) {
		if (hipEventCreateWithFlags(&c.ev[i], hipEventDisableTiming) !=
		    hipSuccess ||
		    hipHostMalloc((void **)&c.h_slab[i], SLAB, 0) != hipSuccess)
			return -1;
	}
	c.pool = new copy_pool(pool_threads());
	c.ready = true;
	return 0;
}

int
grow_dev(uint8_t **p, size_t *cap, size_t want)
{
	if (*cap >= want)
		return 0;
	(void)hipFree(*p);
	*p = NULL;
	*cap = 0;
	if (hipMalloc((void **)p, want) != hipSuccess)
		return -1;
	*cap = want;
	return 0;
}

/* the pieces of host copies that fill bytes [lo, hi) of an image whose
 * segment i (of length len[i]) sits at image offset off[i]; `to_image`
 * picks the direction (host file -> staging slab, or slab -> host file) */
void
slab_pieces(std::vector<piece> &out, uint8_t *slab, size_t lo, size_t hi,
    const std::vector<size_t> &off, const std::vector<size_t> &len,
    const std::vector<uint8_t *> &host, bool to_image)
{
	out.clear();
	/* first segment ending after lo */
	size_t i = std::upper_bound(off.begin(), off.end(), lo) - off.begin();
	i = i > 0 ? i - 1 : 0;
	for (; i < off.size() && off[i] < hi; i++) {
		const size_t a = std::max(lo, off[i]);
		const size_t b = std::min(hi, off[i] + len[i]);
		if (a >= b)
			continue;
		uint8_t *h = host[i] + (a - off[i]);
		uint8_t *s = slab + (a - lo);
		out.push_back(to_image ? piece{ s, h, b - a } :
		    piece{ h, s, b - a });
	}
}

}	/* namespace */

extern "C" int
bjxa__gpu_decode_many(struct bjxa__job *jobs, uint32_t n)
{
	files_ctx &c = ctx;
	std::lock_guard<std::mutex> guard(c.m);
#ifdef XA_FILES_TIMING
	const double t0 = now_ms();
#endif
	if (!bjxa__gpu_present()) {
		errno = ENODEV;
		return -1;
	}
	if (setup(c) < 0) {
		errno = EIO;
		return -1;
	}
	/* device images: inputs at 16-B aligned offsets, outputs packed */
	std::vector<size_t> ioff(n), ilen(n), ooff(n), olen(n);
	std::vector<uint8_t *> isrc(n), odst(n);
	size_t in_total = 0, out_total = 0;
	for (uint32_t i = 0; i < n; i++) {
		ilen[i] = (size_t)(jobs[i].bits * 4 + 1) * jobs[i].ch *
		    jobs[i].eblocks;
		ioff[i] = in_total;
		in_total += (ilen[i] + 15) & ~(size_t)15;
		isrc[i] = (uint8_t *)jobs[i].src;
		ooff[i] = out_total;
		out_total += (size_t)jobs[i].eblocks * 64u * jobs[i].ch;
		odst[i] = (uint8_t *)jobs[i].dst;
	}
	if (grow_dev(&c.d_in, &c.in_cap, in_total + 16) < 0 ||
	    grow_dev(&c.d_out, &c.out_cap, out_total + 16) < 0 ||
	    grow_dev((uint8_t **)&c.d_st, &c.st_cap,
	    (size_t)n * BJXA_HIP_STATUS_WORDS * 4) < 0) {
		errno = ENOMEM;
		return -1;
	}
	std::vector<bjxa_hip_stream_t> hs(n);
	std::vector<uint32_t> st((size_t)n * BJXA_HIP_STATUS_WORDS);
	for (uint32_t i = 0; i < n; i++) {
		memset(&hs[i], 0, sizeof hs[i]);
		hs[i].d_src = c.d_in + ioff[i];
		hs[i].d_dst = c.d_out + ooff[i];
		hs[i].eblocks = jobs[i].eblocks;
		hs[i].frames = (uint64_t)jobs[i].eblocks * 32u;
		hs[i].bits = jobs[i].bits;
		hs[i].channels = jobs[i].ch;
		memcpy(hs[i].state, jobs[i].state, sizeof hs[i].state);
	}
	TMARK("setup");

	/* in: gather slab k while slab k-1 uploads */
	std::vector<piece> pcs;
	bool used[2] = { false, false };
	for (size_t lo = 0, k = 0; lo < in_total; lo += SLAB, k++) {
		const size_t hi = std::min(in_total, lo + SLAB);
		uint8_t *slab = c.h_slab[k & 1];
		if (used[k & 1] && hipEventSynchronize(c.ev[k & 1]) !=
		    hipSuccess)
			goto io;
		slab_pieces(pcs, slab, lo, hi, ioff, ilen, isrc, true);
		c.pool->run(pcs);
		if (hipMemcpyAsync(c.d_in + lo, slab, hi - lo,
		    hipMemcpyHostToDevice, c.stream) != hipSuccess ||
		    hipEventRecord(c.ev[k & 1], c.stream) != hipSuccess)
			goto io;
		used[k & 1] = true;
	}
	TMARK("h2d");
	{
		bjxa_hip_batch_t *b = bjxa__batch_new(hs.data(), n, NULL,
		    c.stream, &c.d_bws, &c.bws_cap);
		if (b == NULL)
			return -1;
		const int r = bjxa_hip_batch_decode_async(b, c.d_st, NULL,
		    c.stream);
		if (r == 0 && (hipMemcpyAsync(st.data(), c.d_st, st.size() * 4,
		    hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
		    hipStreamSynchronize(c.stream) != hipSuccess)) {
			bjxa_hip_batch_free(b);
			goto io;
		}
		bjxa_hip_batch_free(b);
		if (r < 0)
			return -1;
	}
	TMARK("decode");
	/* a stream that failed keeps its PCM before the failing eblock */
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t *w = st.data() + (size_t)i * BJXA_HIP_STATUS_WORDS;
		uint64_t bytes = jobs[i].dst_bytes;
		jobs[i].err_cb = w[XA_ST_ERR];
		if (w[XA_ST_ERR] != 0xffffffffu) {
			const uint64_t cut = (uint64_t)(w[XA_ST_ERR] /
			    jobs[i].ch) * 64u * jobs[i].ch;
			if (bytes > cut)
				bytes = cut;
		}
		olen[i] = bytes;
	}
	/* out: slab k+1 downloads while slab k scatters */
	{
		const size_t nslab = (out_total + SLAB - 1) / SLAB;
		auto fetch = [&](size_t k) {
			const size_t lo = k * SLAB, hi = std::min(out_total,
			    lo + SLAB);
			return hipMemcpyAsync(c.h_slab[k & 1], c.d_out + lo,
			    hi - lo, hipMemcpyDeviceToHost, c.stream) ==
			    hipSuccess && hipEventRecord(c.ev[k & 1],
			    c.stream) == hipSuccess;
		};
		if (nslab > 0 && !fetch(0))
			goto io;
		for (size_t k = 0; k < nslab; k++) {
			if (k + 1 < nslab && !fetch(k + 1))
				goto io;
			if (hipEventSynchronize(c.ev[k & 1]) != hipSuccess)
				goto io;
			const size_t lo = k * SLAB, hi = std::min(out_total,
			    lo + SLAB);
			slab_pieces(pcs, c.h_slab[k & 1], lo, hi, ooff, olen,
			    odst, false);
			c.pool->run(pcs);
		}
	}
	TMARK("d2h");
	return 0;
io:
	(void)hipStreamSynchronize(c.stream);
	errno = EIO;
	return -1;
}
