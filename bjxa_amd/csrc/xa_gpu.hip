/*
 * xa_gpu.hip -- C-ABI around the gfx950 kernels.
 *
 *  - bjxa_hip_* (include/bjxa_hip.h): device-resident entry points.
 *  - bjxa__gpu_* (xa_gpu.h): what the host C library (libbjxa.c) calls from
 *    bjxa_decode()/bjxa_encode() -- the reference's hot-path entries
 *    (src/libbjxa.c:602-661, :759-819) -- to run one call on the GPU.
 *    These are local symbols (libbjxa.map).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <list>
#include <mutex>
#include <thread>
#include <vector>

#include "xa_decode.h"
#include "xa_gpu.h"
#include "xa_pool.h"
#include "../../include/bjxa_hip.h"

#define DEFAULT_WARMUP	8u	/* eblocks; DESIGN.md §3 */
#define MIN_CHUNK	16u
/*
 * Automatic chunking: about target_lanes() chunks -- two resident 256-lane
 * workgroups on each CU of the current device (256 on MI355X), whose
 * memory pipelines bound the speculative kernel.  Uniform chunks of
 * ceil(eblocks / lanes) rounded up to the chunk quantum measured best (C3:
 * 40 eblocks, 489 workgroups; C2: 80).  Plans measured slower and removed
 * (DESIGN.md §3 "Tuning", §5): an exactly balanced one of 512 workgroups
 * with two chunk lengths (12 %), the region kernel K1r (1.7x, R3-2), two
 * chunk lengths per batch stream (R3-8).
 */
#define MAX_DEVICES	64

/* a HIP device is visible; probed once per process, thread-safe */
extern "C" int
bjxa__gpu_present(void)
{
	static std::once_flag once;
	static int present;
	std::call_once(once, [] {
		int n = 0;
		present = hipGetDeviceCount(&n) == hipSuccess && n > 0;
	});
	return present;
}

/* 2 x 256 lanes per CU of the current device (CU count read once per
 * device; 256 CUs if the query fails) */
static uint32_t
target_lanes(void)
{
	static uint32_t cus[MAX_DEVICES];	/* 0 = not read yet */
	int dev = 0, n = 0;
	uint32_t c;

	if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES)
		dev = -1;
	c = dev >= 0 ? __atomic_load_n(&cus[dev], __ATOMIC_RELAXED) : 0;
	if (c == 0) {
		c = (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount,
		    dev < 0 ? 0 : dev) == hipSuccess && n > 0) ? (uint32_t)n : 256u;
		if (dev >= 0)
			__atomic_store_n(&cus[dev], c, __ATOMIC_RELAXED);
	}
	return c * 2u * 256u;
}

/*
 * Tuning variant bit 20: the caller keeps two decodes in flight (two HIP
 * streams, a workspace each).  Plan for one K1 workgroup per CU instead of
 * two: chunks twice as long, so half the warm-up per decoded eblock, and
 * the two launches in flight fill the CUs between them.  Alone such a
 * launch runs at half occupancy.
 */
#define XA_VARIANT_PIPE2	0x100000u

static uint32_t
plan_lanes(const bjxa_hip_tuning_t *t)
{
	const uint32_t lanes = target_lanes();
	return (t && (t->variant & XA_VARIANT_PIPE2)) ? lanes / 2u : lanes;
}

static uint32_t
round_up(uint32_t v, uint32_t m)
{
	return (v + m - 1) / m * m;
}

struct plan {
	uint32_t	C, W;		/* chunk and warm-up, eblocks */
	uint32_t	nchunks;
};

/*
 * Longest chunk: the decode kernel repairs a wave's chunks through one
 * buffer descriptor based at the wave's first eblock, so a wave's 64 chunks
 * of XA (33 B per 8-bit channel block, the largest) must stay under 4 GiB.
 * Only a manual chunk length or a giant batch stream ever gets near it.
 */
static uint32_t
max_chunk(unsigned ch)
{
	const uint32_t G = XA_CHUNK_Q(ch);
	return (uint32_t)((((1ull << 32) - (1ull << 20)) / (64ull * 33u * ch)) /
	    G * G);
}

/* chunk plan for one stream: automatic (above), or tune->chunk eblocks */
static void
plan_chunks(uint32_t eblocks, unsigned ch, const bjxa_hip_tuning_t *t,
    struct plan *p)
{
	const uint32_t G = XA_CHUNK_Q(ch), lanes = plan_lanes(t);
	const uint32_t w = (t && t->warmup >= 0) ? (uint32_t)t->warmup :
	    DEFAULT_WARMUP;
	uint32_t c;
	p->W = round_up(w, G);
	if (t && t->chunk) {
		c = t->chunk;
	} else {
		c = (uint32_t)(((uint64_t)eblocks + lanes - 1) / lanes);
		if (c < MIN_CHUNK)
			c = MIN_CHUNK;
	}
	p->C = round_up(c, G);
	if (p->C > max_chunk(ch))
		p->C = max_chunk(ch);
	p->nchunks = (uint32_t)(((uint64_t)eblocks + p->C - 1) / p->C);
}

/*
 * Pacing of K1 (xa_dec_args::pace): for one stream, the waves of a
 * workgroup meet at a barrier every group when a lane runs at most
 * PACE_MAX_NS super-steps (warm-up included): there (C3: 12, C2: 11) the
 * waves otherwise drift apart and the early finishers leave the tail to
 * fewer requests in flight (spec -3.8 % / -3.5 %).  Batches only up to
 * PACE_MAX_NS_BATCH: C3's 5M eblocks as 16 or 64 streams (NS 11-12) gain
 * 4.5 % / 1.1 % paced, while C5g (NS 18), C4 (NS 26) and C5 (NS 130) gain
 * nothing or lose 1-3 % (interleaved A/B).  Tuning variant
 * bits 8-11 override: 15 = off, 1-14 = barrier every that many groups.
 */
#define PACE_MAX_NS	32u
#define PACE_MAX_NS_BATCH	12u

static uint32_t
pick_pace(uint32_t ns, bool batch, const bjxa_hip_tuning_t *t)
{
	const uint32_t code = t ? (t->variant >> 8) & 15u : 0u;
	if (code == 15u)
		return 0u;
	if (code != 0u)
		return code;
	return ns <= (batch ? PACE_MAX_NS_BATCH : PACE_MAX_NS) ? 1u : 0u;
}

/* workspace layout: control words, g[n], e[n], the queue (2n entries: a
 * chunk may be queued twice, as a late boundary and after a cascade), then
 * one 16-B exit record per wave */
/* the verify pass's test knobs (tuning variant bits 18, 19) */
#define XA_VARIANT_NORECORD	0x40000u
#define XA_VARIANT_NOWAIT	0x80000u

static void
verify_knobs(const bjxa_hip_tuning_t *t, uint32_t *spin, uint32_t *flags)
{
	const uint32_t v = t ? t->variant : 0u;
	*spin = (v & XA_VARIANT_NOWAIT) ? 0u : XA_SPIN_TICKS;
	*flags = (v & XA_VARIANT_NORECORD) ? XA_F_NORECORD : 0u;
}

static size_t
ws_exits_off(uint32_t nchunks)
{
	return (XA_CTL_WORDS * 4 + (size_t)nchunks * (8 + 8 + 8) + 15) &
	    ~(size_t)15;
}

static size_t
ws_bytes(uint32_t nchunks)
{
	return ws_exits_off(nchunks) + (size_t)(nchunks + 63) / 64 * 16 + 64;
}

/*
 * The exit records are recognised by their launch tag alone (xa_decode.hip
 * put_exit/get_exit).  The tag is a small counter, so the record region must
 * not hold words another use of the memory left behind: the g/e states and
 * queue entries of a decode with another layout (a smaller stream in a
 * workspace sized for a larger one puts its records on them) are small
 * integers too, and a stale pair equal to the tag would pass as the wave
 * before's exit.  After bjxa_hip_workspace_init the region is zero, and it
 * stays records while the workspace keeps its layout; a decode whose record
 * region differs from the last one on the same workspace zeroes its region
 * first (a stream-ordered memset of 16 B per wave).  Remembered per
 * workspace address; a workspace this table has forgotten is zeroed too.
 */
#define WS_SEEN		64
#define WS_ZEROED	((size_t)-1)	/* whole workspace zero (just initialised) */

static std::mutex ws_seen_mu;
static struct {
	const void	*ws;
	size_t		off;		/* record region: byte offset, length */
	size_t		len;
} ws_seen[WS_SEEN];
static unsigned ws_seen_next;

/* record that workspace ws now has its records at [off, off + len); true if
 * that region may hold words of another layout (it must be zeroed) */
static bool
ws_records_stale(const void *ws, size_t off, size_t len)
{
	std::lock_guard<std::mutex> lk(ws_seen_mu);
	for (unsigned i = 0; i < WS_SEEN; i++) {
		if (ws_seen[i].ws != ws)
			continue;
		const bool same = ws_seen[i].off == WS_ZEROED ||
		    (ws_seen[i].off == off && ws_seen[i].len == len);
		ws_seen[i].off = off;
		ws_seen[i].len = len;
		return !same;
	}
	const unsigned i = ws_seen_next++ % WS_SEEN;
	ws_seen[i].ws = ws;
	ws_seen[i].off = off;
	ws_seen[i].len = len;
	return true;
}

static void
ws_records_zeroed(const void *ws)
{
	std::lock_guard<std::mutex> lk(ws_seen_mu);
	for (unsigned i = 0; i < WS_SEEN; i++)
		if (ws_seen[i].ws == ws) {
			ws_seen[i].off = WS_ZEROED;
			return;
		}
	const unsigned i = ws_seen_next++ % WS_SEEN;
	ws_seen[i].ws = ws;
	ws_seen[i].off = WS_ZEROED;
	ws_seen[i].len = 0;
}

extern "C" size_t
bjxa_hip_decode_workspace(uint32_t eblocks, unsigned channels,
    const bjxa_hip_tuning_t *tune)
{
	struct plan p;
	if (channels != 1 && channels != 2)
		return 0;
	plan_chunks(eblocks, channels, tune, &p);
	uint64_t n = p.nchunks;
	if (!(tune && tune->chunk)) {
		/*
		 * The automatic plan is not monotone in the stream length (C3's
		 * 5,000,000 eblocks plan 125,000 chunks of 40, 2,600,000 plan
		 * 130,000 of 20), but no stream of at most `eblocks` plans more
		 * than min(ceil(eblocks / MIN_CHUNK), lanes) chunks: sized for
		 * that, the workspace serves every shorter stream too
		 * (INTEGRATION.md), for at most 24 B per chunk more.
		 */
		const uint64_t b = std::min(((uint64_t)eblocks + MIN_CHUNK - 1) /
		    MIN_CHUNK, (uint64_t)plan_lanes(tune));
		n = std::max(n, b);
	}
	return ws_bytes((uint32_t)n);
}

__global__ void
xa_ws_init(uint32_t *ctl)
{
	if (threadIdx.x < XA_CTL_WORDS)
		ctl[threadIdx.x] = threadIdx.x == XA_CTL_ERR ? 0xffffffffu : 0u;
}

extern "C" int
bjxa_hip_workspace_init(void *d_ws, size_t ws_len, void *stream)
{
	if (d_ws == NULL || ws_len < XA_CTL_WORDS * 4) {
		errno = EINVAL;
		return -1;
	}
	if (!bjxa__gpu_present()) {
		errno = ENODEV;
		return -1;
	}
	/* all of it: no exit record of an earlier user of the memory survives
	 * (records of this process's earlier launches carry other tags) */
	if (hipMemsetAsync(d_ws, 0, ws_len, (hipStream_t)stream) != hipSuccess) {
		errno = EIO;
		return -1;
	}
	hipLaunchKernelGGL(xa_ws_init, dim3(1), dim3(64), 0,
	    (hipStream_t)stream, (uint32_t *)d_ws);
	if (hipGetLastError() != hipSuccess) {
		errno = EIO;
		return -1;
	}
	ws_records_zeroed(d_ws);
	return 0;
}

/* bjxa_hip_decode_async, with the entry state optionally read on the
 * device from an earlier decode's status words (init_dev, stream order) */
static int
decode_async(const bjxa_hip_stream_t *s, void *d_ws, size_t ws_len,
    uint32_t *d_status, const bjxa_hip_tuning_t *tune, void *stream,
    const uint32_t *init_dev)
{
	struct plan p;
	if (s == NULL || d_ws == NULL || d_status == NULL || s->d_src == NULL ||
	    s->d_dst == NULL || (s->bits != 4 && s->bits != 6 && s->bits != 8) ||
	    (s->channels != 1 && s->channels != 2) || s->eblocks == 0 ||
	    s->frames > (uint64_t)s->eblocks * 32u ||
	    s->frames <= (uint64_t)(s->eblocks - 1) * 32u ||
	    ((uintptr_t)s->d_src & 3u) != 0 || ((uintptr_t)s->d_dst & 15u) != 0 ||
	    ((uintptr_t)d_ws & 15u) != 0) {
		errno = EINVAL;
		return -1;
	}
	if (!bjxa__gpu_present()) {
		errno = ENODEV;
		return -1;
	}
	plan_chunks(s->eblocks, s->channels, tune, &p);
	xa_dec_args a;
	a.src = (const uint8_t *)s->d_src;
	a.dst = (uint8_t *)s->d_dst;
	a.pcm_bytes = s->frames * 2u * s->channels;
	a.eblocks = s->eblocks;
	a.nchunks = p.nchunks;
	a.C = p.C;
	a.W = p.W;
	a.pace = pick_pace((p.W + p.C) / XA_CHUNK_Q(s->channels), false, tune);
	a.init[0] = ((uint32_t)(uint16_t)s->state[0]) |
	    ((uint32_t)(uint16_t)s->state[1] << 16);
	a.init[1] = ((uint32_t)(uint16_t)s->state[2]) |
	    ((uint32_t)(uint16_t)s->state[3] << 16);
	a.init_dev = init_dev;
	if (ws_len < ws_bytes(p.nchunks)) {
		errno = EINVAL;
		return -1;
	}
	uint8_t *ws = (uint8_t *)d_ws;
	a.ctl = (uint32_t *)ws;
	a.g = (uint2 *)(ws + XA_CTL_WORDS * 4);
	a.e = a.g + p.nchunks;
	a.queue = (uint32_t *)(a.e + p.nchunks);
	a.nq = &a.ctl[XA_CTL_NQ];
	a.qcap = 2u * p.nchunks;
	a.qbase = 0;
	a.ovf = &a.ctl[XA_CTL_OVF];
	a.exits = (uint4 *)(ws + ws_exits_off(p.nchunks));
	a.tag = 0;	/* set per launch */
	verify_knobs(tune, &a.spin, &a.flags);
	a.status = d_status;
	const size_t xlen = (size_t)(p.nchunks + 63) / 64 * 16;
	if (ws_records_stale(d_ws, ws_exits_off(p.nchunks), xlen) &&
	    hipMemsetAsync(a.exits, 0, xlen, (hipStream_t)stream) != hipSuccess) {
		(void)hipGetLastError();
		(void)ws_records_stale(d_ws, 0, 0);	/* no region: zero next time */
		errno = EIO;
		return -1;
	}
	hipEvent_t e0 = tune ? (hipEvent_t)tune->ev_spec[0] : NULL;
	hipEvent_t e1 = tune ? (hipEvent_t)tune->ev_spec[1] : NULL;
	const hipError_t rc = xa_decode_launch(a, s->bits, s->channels,
	    (hipStream_t)stream, e0, e1);
	if (rc != hipSuccess) {
		/* the first kernel may have run without the tail that resets
		 * the control words: leave the workspace initialised again */
		(void)hipGetLastError();
		(void)bjxa_hip_workspace_init(d_ws, ws_len, stream);
		errno = EIO;
		return -1;
	}
	return 0;
}

extern "C" int
bjxa_hip_decode_async(const bjxa_hip_stream_t *s, void *d_ws, size_t ws_len,
    uint32_t *d_status, const bjxa_hip_tuning_t *tune, void *stream)
{
	return decode_async(s, d_ws, ws_len, d_status, tune, stream, NULL);
}

extern "C" int
bjxa_hip_encode_async(const void *d_pcm, uint64_t frames, unsigned bits,
    unsigned channels, void *d_xa, void *stream)
{
	if (d_pcm == NULL || d_xa == NULL || frames == 0 ||
	    (bits != 4 && bits != 6 && bits != 8) ||
	    (channels != 1 && channels != 2) || (frames + 31) / 32 > 0xffffffffu ||
	    ((uintptr_t)d_pcm & 15u) != 0 || ((uintptr_t)d_xa & 3u) != 0) {
		errno = EINVAL;
		return -1;
	}
	if (!bjxa__gpu_present()) {
		errno = ENODEV;
		return -1;
	}
	xa_enc_args a;
	a.src = (const uint8_t *)d_pcm;
	a.dst = (uint8_t *)d_xa;
	a.frames = frames;
	a.eblocks = (uint32_t)((frames + 31) / 32);
	if (xa_encode_launch(a, bits, channels, (hipStream_t)stream) !=
	    hipSuccess) {
		errno = EIO;
		return -1;
	}
	return 0;
}

/* ------------------------------------------------------------------ */
/* batched decode (bjxa_hip_batch_*)                                    */

struct bjxa_hip_batch {
	void		*d_ws;
	bool		owns_ws;	/* false: a workspace lent by the caller */
	bool		launched;	/* `done` has been recorded */
	hipEvent_t	done;		/* after the last decode's kernels */
	xa_batch_args	args;
};

/* round x up to a multiple of 64 bytes */
static size_t
al64(size_t x)
{
	return (x + 63) & ~(size_t)63;
}

__global__ void
xa_batch_init(uint32_t *ctl, uint32_t *sctl, uint32_t n)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (blockIdx.x == 0 && threadIdx.x < XA_CTL_WORDS)
		ctl[threadIdx.x] = 0;
	if (i < n) {
		sctl[i * XA_SCTL_WORDS + XA_SCTL_ERR] = 0xffffffffu;
		sctl[i * XA_SCTL_WORDS + XA_SCTL_TAIL] = 0;
		sctl[i * XA_SCTL_WORDS + XA_SCTL_FIXED] = 0;
		sctl[i * XA_SCTL_WORDS + 3] = 0;
	}
}

static int
stream_ok(const bjxa_hip_stream_t *s)
{
	return s->d_src != NULL && s->d_dst != NULL &&
	    (s->bits == 4 || s->bits == 6 || s->bits == 8) &&
	    (s->channels == 1 || s->channels == 2) && s->eblocks != 0 &&
	    s->frames <= (uint64_t)s->eblocks * 32u &&
	    s->frames > (uint64_t)(s->eblocks - 1) * 32u &&
	    ((uintptr_t)s->d_src & 3u) == 0 && ((uintptr_t)s->d_dst & 15u) == 0;
}

/*
 * Streams whose PCM images are carved out of one large device allocation
 * (as bjxa_hip_decode_files does, or a caller packing a batch into one
 * buffer) decode slower when their chunk length puts the lanes' PCM 8 KiB
 * apart: C5's per-GPU share at 8 GPUs (64 eblocks = 8 KiB) runs 0.43 ms
 * packed against 0.30 ms in allocations of their own, whatever the VA gaps
 * between the streams (DESIGN.md §5 round 2 exp. 14, R3-7, R4-11).  Why is
 * not settled: one hypothesis is that one physically contiguous run puts
 * every lane of every stream on the same HBM channels, but a store-only
 * probe pays the 8 KiB stride in both layouts.  Such
 * streams get chunks one quantum longer.  Streams in allocations of their
 * own do not pay the penalty, and there the longer chunks only cost time
 * (round 2 exp. 16), so the planner asks the runtime which allocation each
 * PCM image belongs to and lengthens the chunks of streams that share an
 * allocation of at least XA_PACKED_SPAN bytes with at least XA_PACKED_MIN - 1
 * others.  The span keeps out a caching allocator's shared segments: torch
 * carves mid-size tensors out of 20 MiB segments, and 512 streams of 2 MiB
 * PCM so placed (ten to a segment) run 0.3187 ms at 64-eblock chunks
 * against 0.3477 at 68; an 8 KiB lane stride only
 * arises for batches of ~1 GiB of PCM on 256 CUs, so an allocation that
 * holds eight such images and reaches 64 MiB is the caller's own.  Tuning
 * variant bit 16 forces the longer chunks for every stream, bit 17 forbids
 * them.
 */
#define XA_VARIANT_DECOR	0x10000u
#define XA_VARIANT_NODECOR	0x20000u
#define XA_PACKED_MIN		8u
#define XA_PACKED_SPAN		(64ull << 20)

struct pcm_base {
	uintptr_t	base;	/* the allocation holding the PCM image */
	uint32_t	idx;
};

static int
by_base(const void *x, const void *y)
{
	const struct pcm_base *a = (const struct pcm_base *)x;
	const struct pcm_base *b = (const struct pcm_base *)y;
	if (a->base != b->base)
		return a->base < b->base ? -1 : 1;
	return a->idx < b->idx ? -1 : (a->idx > b->idx);
}

/*
 * packed[i] = 1 for the streams whose PCM shares an allocation of at least
 * XA_PACKED_SPAN bytes with at least XA_PACKED_MIN - 1 others (or all / none
 * under the tuning bits).
 * Returns a calloc'ed array of n flags, or NULL with errno ENOMEM.  The
 * runtime's error state is cleared after an address it cannot place (that
 * error is not the caller's).
 */
static uint8_t *
packed_pcm(const bjxa_hip_stream_t *s, uint32_t n, const bjxa_hip_tuning_t *t)
{
	const uint32_t v = t ? t->variant : 0u;
	uint8_t *packed = (uint8_t *)calloc(n, 1);
	if (packed == NULL) {
		errno = ENOMEM;
		return NULL;
	}
	if (v & XA_VARIANT_DECOR)
		memset(packed, 1, n);
	if (v & (XA_VARIANT_DECOR | XA_VARIANT_NODECOR) || n < XA_PACKED_MIN)
		return packed;
	struct pcm_base *base = (struct pcm_base *)calloc(n, sizeof *base);
	if (base == NULL) {
		free(packed);
		errno = ENOMEM;
		return NULL;
	}
	bool failed = false;
	for (uint32_t i = 0; i < n; i++) {
		hipDeviceptr_t b = NULL;
		size_t sz = 0;
		if (hipMemGetAddressRange(&b, &sz, (hipDeviceptr_t)s[i].d_dst) !=
		    hipSuccess) {
			b = NULL;	/* not a device allocation we can see */
			failed = true;
		} else if (sz < XA_PACKED_SPAN) {
			b = NULL;	/* a small allocation: never "packed" */
		}
		base[i].base = (uintptr_t)b;
		base[i].idx = i;
	}
	if (failed)
		(void)hipGetLastError();
	qsort(base, n, sizeof *base, by_base);
	for (uint32_t i = 0; i < n;) {
		uint32_t j = i;
		while (j < n && base[j].base == base[i].base)
			j++;
		if (base[i].base != 0 && j - i >= XA_PACKED_MIN)
			for (uint32_t k = i; k < j; k++)
				packed[base[k].idx] = 1;
		i = j;
	}
	free(base);
	return packed;
}

/*
 * Plan: one budget of channel blocks per lane, Cb = the batch's channel
 * blocks / target_lanes() (at least MIN_CHUNK, a multiple of 4); a stream of
 * E eblocks and ch channels gets k = round(E*ch / (64*Cb)) >= 1 whole
 * waves and chunks of ceil(E / 64k) eblocks (rounded up to its group, at
 * least MIN_CHUNK), so a stereo lane decodes about Cb/2 eblocks and a mono
 * lane about Cb blocks -- the single-stream optimum (C3: 40, C2: 80).
 */
extern "C" bjxa_hip_batch_t *
bjxa_hip_batch_new(const bjxa_hip_stream_t *s, uint32_t n,
    const bjxa_hip_tuning_t *tune, void *stream)
{
	return bjxa__batch_new(s, n, tune, stream, NULL, NULL);
}

/*
 * bjxa_hip_batch_new, optionally in a workspace the caller keeps across
 * batches (*ws_cache of *ws_cap bytes, grown here when too small; the
 * batch then does not free it).  The files path uses this so that a call
 * does not allocate and free device memory.
 */
extern "C" bjxa_hip_batch_t *
bjxa__batch_new(const bjxa_hip_stream_t *s, uint32_t n,
    const bjxa_hip_tuning_t *tune, void *stream, void **ws_cache,
    size_t *ws_cap)
{
	if (s == NULL || n == 0) {
		errno = EINVAL;
		return NULL;
	}
	uint64_t cblocks = 0;
	for (uint32_t i = 0; i < n; i++) {
		if (!stream_ok(&s[i])) {
			errno = EINVAL;
			return NULL;
		}
		cblocks += (uint64_t)s[i].eblocks * s[i].channels;
	}
	if (!bjxa__gpu_present()) {
		errno = ENODEV;
		return NULL;
	}
	const uint32_t lanes = plan_lanes(tune);
	uint64_t cb = (cblocks + lanes - 1) / lanes;
	if (tune && tune->chunk)
		cb = tune->chunk;
	if (cb < MIN_CHUNK)
		cb = MIN_CHUNK;
	cb = (cb + 3) & ~(uint64_t)3;
	const uint32_t w = (tune && tune->warmup >= 0) ? (uint32_t)tune->warmup :
	    DEFAULT_WARMUP;
	const uint32_t W = (w + 7) & ~7u;	/* a whole chunk quantum of every format */

	uint8_t *packed = packed_pcm(s, n, tune);
	if (packed == NULL)
		return NULL;
	xa_batch_stream *hs = (xa_batch_stream *)calloc(n, sizeof *hs);
	if (hs == NULL) {
		free(packed);
		errno = ENOMEM;
		return NULL;
	}
	uint64_t nwaves = 0;
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t E = s[i].eblocks, ch = s[i].channels,
		    G = XA_CHUNK_Q(ch);
		uint64_t k = ((uint64_t)E * ch + 32 * cb) / (64 * cb);
		if (k == 0)
			k = 1;
		uint64_t c = (E + 64 * k - 1) / (64 * k);
		if (c > max_chunk(ch)) {
			/* more waves, so that a wave's XA stays under 4 GiB */
			k = (E + 64ull * max_chunk(ch) - 1) / (64ull * max_chunk(ch));
			c = (E + 64 * k - 1) / (64 * k);
		}
		if (c < MIN_CHUNK)
			c = MIN_CHUNK;
		c = (c + G - 1) / G * G;
		if (packed[i] && (c * 64u * ch) % 8192u == 0)
			c += G;
		const uint32_t nch = (uint32_t)((E + c - 1) / c);
		hs[i].src = (const uint8_t *)s[i].d_src;
		hs[i].dst = (uint8_t *)s[i].d_dst;
		hs[i].pcm_bytes = s[i].frames * 2u * ch;
		hs[i].eblocks = E;
		hs[i].nchunks = nch;
		hs[i].cbase = (uint32_t)(64 * nwaves);
		hs[i].C = (uint32_t)c;
		hs[i].init[0] = ((uint32_t)(uint16_t)s[i].state[0]) |
		    ((uint32_t)(uint16_t)s[i].state[1] << 16);
		hs[i].init[1] = ((uint32_t)(uint16_t)s[i].state[2]) |
		    ((uint32_t)(uint16_t)s[i].state[3] << 16);
		hs[i].fmt = s[i].bits | ch << 8;
		nwaves += (nch + 63) / 64;
	}
	free(packed);
	if (64 * nwaves > 0x7fffffffu) {
		free(hs);
		errno = EINVAL;
		return NULL;
	}
	uint32_t *hw = (uint32_t *)malloc(nwaves * 4);
	bjxa_hip_batch_t *b = (bjxa_hip_batch_t *)calloc(1, sizeof *b);
	if (hw == NULL || b == NULL) {
		free(hs);
		free(hw);
		free(b);
		errno = ENOMEM;
		return NULL;
	}
	for (uint32_t i = 0, wv = 0; i < n; i++)
		for (uint32_t j = 0; j < (hs[i].nchunks + 63) / 64; j++)
			hw[wv++] = i;

	const size_t nc = 64 * nwaves;
	const size_t o_sctl = al64(XA_CTL_WORDS * 4);
	const size_t o_str = o_sctl + al64((size_t)n * XA_SCTL_WORDS * 4);
	const size_t o_wav = o_str + al64((size_t)n * sizeof(xa_batch_stream));
	const size_t o_g = o_wav + al64(nwaves * 4);
	const size_t o_e = o_g + nc * 8;
	const size_t o_q = o_e + nc * 8;
	const size_t o_x = al64(o_q + 2 * nc * 4);	/* exit records */
	const size_t len = o_x + nwaves * 16;
	uint8_t *ws = NULL;
	if (ws_cache != NULL && *ws_cap >= len) {
		ws = (uint8_t *)*ws_cache;
	} else {
		if (ws_cache != NULL) {
			/* the previous user of the cache has completed */
			(void)hipStreamSynchronize((hipStream_t)stream);
			(void)hipFree(*ws_cache);
			*ws_cache = NULL;
			*ws_cap = 0;
		}
		if (hipMalloc((void **)&ws, len) != hipSuccess) {
			free(hs);
			free(hw);
			free(b);
			errno = ENOMEM;
			return NULL;
		}
		if (ws_cache != NULL) {
			*ws_cache = ws;
			*ws_cap = len;
		}
	}
	b->d_ws = ws;
	b->owns_ws = ws_cache == NULL;
	if (hipEventCreateWithFlags(&b->done, hipEventDisableTiming) !=
	    hipSuccess) {
		if (b->owns_ws)
			(void)hipFree(ws);
		free(hs);
		free(hw);
		free(b);
		errno = EIO;
		return NULL;
	}
	xa_batch_args &a = b->args;
	a.streams = (const xa_batch_stream *)(ws + o_str);
	a.wstream = (const uint32_t *)(ws + o_wav);
	a.nstreams = n;
	a.nwaves = (uint32_t)nwaves;
	a.W = W;
	/* super-steps of a lane: its channel blocks (warm-up included) over
	 * the 8 per super-step, the same for every format */
	a.pace = pick_pace((uint32_t)((a.W * 2u + cb) / 8u), true, tune);
	a.g = (uint2 *)(ws + o_g);
	a.e = (uint2 *)(ws + o_e);
	a.queue = (uint32_t *)(ws + o_q);
	a.exits = (uint4 *)(ws + o_x);
	a.tag = 0;	/* set per launch */
	verify_knobs(tune, &a.spin, &a.flags);
	a.ctl = (uint32_t *)ws;
	a.sctl = (uint32_t *)(ws + o_sctl);
	a.status = NULL;
	/* stream-ordered uploads: the workspace may still be in use by an
	 * earlier batch on the same stream (the files path) */
	int bad = hipMemcpyAsync(ws + o_str, hs, (size_t)n * sizeof *hs,
	    hipMemcpyHostToDevice, (hipStream_t)stream) != hipSuccess ||
	    hipMemcpyAsync(ws + o_wav, hw, nwaves * 4, hipMemcpyHostToDevice,
	    (hipStream_t)stream) != hipSuccess ||
	    hipStreamSynchronize((hipStream_t)stream) != hipSuccess;
	free(hs);
	free(hw);
	if (!bad)
		bad = hipMemsetAsync(ws + o_x, 0, nwaves * 16, (hipStream_t)stream) !=
		    hipSuccess;
	if (!bad) {
		hipLaunchKernelGGL(xa_batch_init, dim3((n + 255) / 256), dim3(256),
		    0, (hipStream_t)stream, a.ctl, a.sctl, n);
		bad = hipGetLastError() != hipSuccess;
	}
	if (bad) {
		(void)hipEventDestroy(b->done);
		if (b->owns_ws)
			(void)hipFree(ws);
		free(b);
		errno = EIO;
		return NULL;
	}
	return b;
}

extern "C" int
bjxa_hip_batch_decode_async(bjxa_hip_batch_t *b, uint32_t *d_status,
    const bjxa_hip_tuning_t *tune, void *stream)
{
	if (b == NULL || d_status == NULL) {
		errno = EINVAL;
		return -1;
	}
	b->args.status = d_status;
	if (xa_decode_batch_launch(b->args, (hipStream_t)stream,
	    tune ? (hipEvent_t)tune->ev_spec[0] : NULL,
	    tune ? (hipEvent_t)tune->ev_spec[1] : NULL) != hipSuccess) {
		/* the first kernel may have run without the tail that resets
		 * the control words: reset them for the next decode */
		(void)hipGetLastError();
		hipLaunchKernelGGL(xa_batch_init, dim3((b->args.nstreams + 255) /
		    256), dim3(256), 0, (hipStream_t)stream, b->args.ctl,
		    b->args.sctl, b->args.nstreams);
		(void)hipGetLastError();
		errno = EIO;
		return -1;
	}
	if (hipEventRecord(b->done, (hipStream_t)stream) != hipSuccess) {
		errno = EIO;
		return -1;
	}
	b->launched = true;
	return 0;
}

/* waits for the batch's own last decode only (not the whole device) */
extern "C" void
bjxa_hip_batch_free(bjxa_hip_batch_t *b)
{
	if (b == NULL)
		return;
	if (b->launched)
		(void)hipEventSynchronize(b->done);
	(void)hipEventDestroy(b->done);
	if (b->owns_ws)
		(void)hipFree(b->d_ws);
	free(b);
}

extern "C" const char *
bjxa_hip_version(void)
{
	return "bjxa-mi355x 0.2 gfx950 (spec/fix decode, batched decode, group encode)";
}

/* ------------------------------------------------------------------ */
/* per-codec GPU context behind bjxa_decode()/bjxa_encode()            */

struct bjxa__gpu {
	int		device;		/* current HIP device at creation */
	hipStream_t	stream;
	void		*d_in, *d_out, *d_ws;
	size_t		in_cap, out_cap, ws_cap;
	uint8_t		*h_small;	/* pinned: small-call in | out | status */
	uint8_t		*d_small;	/* its device view */
	uint32_t	*d_status;
	bool		ws_stale;	/* a call failed: initialise the
					 * workspace again before the next */
	/* the duplex route of large calls (duplex_decode), made on first use */
	hipStream_t	s_out, s_dec;
	uint8_t		*h_stage;	/* pinned: DUPLEX_SLOTS staging slots */
	uint8_t		*d_stage;	/* its device view */
	uint32_t	*d_sst;		/* per-slab status words */
	uint32_t	*h_hst;		/* pinned: per-slab status for the host
					 * (direct route) */
	uint32_t	*d_hst;		/* its device view */
	size_t		sst_cap;	/* in slabs */
	hipEvent_t	*evp;		/* the route's events, kept across calls */
	size_t		evp_n;
};

static int
grow(void **p, size_t *cap, size_t need)
{
	if (*cap >= need)
		return 0;
	if (*p != NULL)
		(void)hipFree(*p);
	*p = NULL;
	*cap = 0;
	need = (need + 4095) & ~(size_t)4095;
	if (hipMalloc(p, need) != hipSuccess) {
		*p = NULL;
		errno = ENOMEM;
		return -1;
	}
	*cap = need;
	return 0;
}

/*
 * A codec is bound to the HIP device that is current on the thread that
 * first runs it on the GPU; every later call switches the calling thread
 * to that device for the call's duration and back (so a codec created
 * under hipSetDevice(k) keeps using GPU k from any thread).
 */
struct device_scope {
	int	prev;
	bool	moved;
	explicit device_scope(int dev) : prev(-1), moved(false)
	{
		if (hipGetDevice(&prev) == hipSuccess && prev != dev)
			moved = hipSetDevice(dev) == hipSuccess;
	}
	~device_scope()
	{
		if (moved)
			(void)hipSetDevice(prev);
	}
};

extern "C" struct bjxa__gpu *
bjxa__gpu_new(void)
{
	if (!bjxa__gpu_present()) {
		errno = ENODEV;
		return NULL;
	}
	struct bjxa__gpu *g = (struct bjxa__gpu *)calloc(1, sizeof *g);
	if (g == NULL) {
		errno = ENOMEM;
		return NULL;
	}
	if (hipGetDevice(&g->device) != hipSuccess)
		g->device = 0;
	if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) !=
	    hipSuccess || hipMalloc((void **)&g->d_status, 64) != hipSuccess) {
		free(g);
		errno = ENODEV;
		return NULL;
	}
	return g;
}

extern "C" void
bjxa__gpu_free(struct bjxa__gpu *g)
{
	if (g == NULL)
		return;
	device_scope on(g->device);
	(void)hipStreamSynchronize(g->stream);
	(void)hipFree(g->d_in);
	(void)hipFree(g->d_out);
	(void)hipFree(g->d_ws);
	(void)hipFree(g->d_status);
	if (g->h_small != NULL)
		(void)hipHostFree(g->h_small);
	if (g->s_out != NULL) {
		(void)hipStreamSynchronize(g->s_out);
		(void)hipStreamSynchronize(g->s_dec);
		(void)hipStreamDestroy(g->s_out);
		(void)hipStreamDestroy(g->s_dec);
	}
	if (g->h_stage != NULL)
		(void)hipHostFree(g->h_stage);
	(void)hipFree(g->d_sst);
	if (g->h_hst != NULL)
		(void)hipHostFree(g->h_hst);
	for (size_t i = 0; i < g->evp_n; i++)
		(void)hipEventDestroy(g->evp[i]);
	free(g->evp);
	(void)hipStreamDestroy(g->stream);
	free(g);
}

static int
io_fail(void)
{
	errno = EIO;
	return -1;
}

static int
small_buffer(struct bjxa__gpu *g)
{
	if (g->h_small != NULL)
		return 0;
	if (hipHostMalloc((void **)&g->h_small, XA_SMALL_BYTES,
	    hipHostMallocDefault) != hipSuccess) {
		g->h_small = NULL;
		errno = ENOMEM;
		return -1;
	}
	if (hipHostGetDevicePointer((void **)&g->d_small, g->h_small, 0) !=
	    hipSuccess) {
		(void)hipHostFree(g->h_small);
		g->h_small = NULL;
		errno = EIO;
		return -1;
	}
	return 0;
}

/* at most XA_SMALL_MAX eblocks: one launch over the pinned buffer */
static int
small_decode(struct bjxa__gpu *g, const void *src, uint32_t eblocks,
    unsigned bits, unsigned ch, int16_t state[4], void *dst,
    uint64_t dst_bytes, uint32_t *err_cb)
{
	const size_t in_bytes = (size_t)(bits * 4 + 1) * ch * eblocks;
	uint32_t init[2];

	if (small_buffer(g) < 0)
		return -1;
	memcpy(g->h_small, src, in_bytes);
	init[0] = ((uint32_t)(uint16_t)state[0]) |
	    ((uint32_t)(uint16_t)state[1] << 16);
	init[1] = ((uint32_t)(uint16_t)state[2]) |
	    ((uint32_t)(uint16_t)state[3] << 16);
	if (xa_small_decode_launch(g->d_small, g->d_small + XA_SMALL_IN, eblocks,
	    bits, ch, init, g->stream) != hipSuccess ||
	    hipStreamSynchronize(g->stream) != hipSuccess)
		return io_fail();
	const volatile uint32_t *st = (const volatile uint32_t *)(g->h_small +
	    XA_SMALL_IN + XA_SMALL_STATUS);
	*err_cb = st[0];
	if (st[0] != 0xffffffffu && dst_bytes > (uint64_t)(st[0] / ch) * 64u * ch)
		dst_bytes = (uint64_t)(st[0] / ch) * 64u * ch;
	state[0] = (int16_t)(st[1] & 0xffffu);
	state[1] = (int16_t)(st[1] >> 16);
	state[2] = (int16_t)(st[2] & 0xffffu);
	state[3] = (int16_t)(st[2] >> 16);
	memcpy(dst, g->h_small + XA_SMALL_IN, dst_bytes);
	return 0;
}

/*
 * The state at a failing eblock j (bad channel bad_c) of the PCM in g->d_out:
 * the decode stops before eblock j, as the reference does; the left channel
 * of that eblock is already advanced if the right block is the bad one
 * (src/libbjxa.c:633-643).
 */
static int
err_state(struct bjxa__gpu *g, uint32_t j, uint32_t bad_c, unsigned ch,
    int16_t state[4])
{
	int16_t fr[2][2];	/* frames 30, 31 */
	if (j > 0) {
		if (hipMemcpy(fr, (uint8_t *)g->d_out + ((size_t)j * 64u * ch) -
		    4u * ch, 4u * ch, hipMemcpyDeviceToHost) != hipSuccess)
			return io_fail();
		for (unsigned c = 0; c < ch; c++) {
			state[2 * c] = ch == 2 ? fr[1][c] : ((int16_t *)fr)[1];
			state[2 * c + 1] = ch == 2 ? fr[0][c] : ((int16_t *)fr)[0];
		}
	}
	if (ch == 2 && bad_c == 1) {
		if (hipMemcpy(fr, (uint8_t *)g->d_out + ((size_t)(j + 1) * 128u) -
		    8u, 8u, hipMemcpyDeviceToHost) != hipSuccess)
			return io_fail();
		state[0] = fr[1][0];
		state[1] = fr[0][0];
	}
	return 0;
}

static void
exit_state(const uint32_t *st, int16_t state[4])
{
	state[0] = (int16_t)(st[XA_ST_STATE_L] & 0xffffu);
	state[1] = (int16_t)(st[XA_ST_STATE_L] >> 16);
	state[2] = (int16_t)(st[XA_ST_STATE_R] & 0xffffu);
	state[3] = (int16_t)(st[XA_ST_STATE_R] >> 16);
}

/* the codec's device buffers for a call of `eblocks` (inputs, PCM, and a
 * workspace for decodes of up to `ws_eblocks`), the workspace initialised
 * when new or left stale by a failed call */
static int
call_buffers(struct bjxa__gpu *g, uint32_t eblocks, uint32_t ws_eblocks,
    unsigned bits, unsigned ch)
{
	const size_t in_bytes = (size_t)(bits * 4 + 1) * ch * eblocks;
	const size_t out_full = (size_t)eblocks * 64u * ch;
	int fresh = g->d_ws == NULL || g->ws_stale;
	const size_t wsn = bjxa_hip_decode_workspace(ws_eblocks, ch, NULL);
	if (grow(&g->d_in, &g->in_cap, in_bytes + 16) < 0 ||
	    grow(&g->d_out, &g->out_cap, out_full) < 0)
		return -1;
	if (g->ws_cap < wsn) {
		if (grow(&g->d_ws, &g->ws_cap, wsn) < 0)
			return -1;
		fresh = 1;
	}
	if (fresh && bjxa_hip_workspace_init(g->d_ws, g->ws_cap, g->stream) < 0)
		return -1;
	return 0;
}

/*
 * ------------------------------------------------------------------
 * Large host-pointer calls with both PCIe directions busy at once
 * (DESIGN.md §5 R6-7).  The copy engines do not overlap an H2D with a D2H
 * (the 2M-eblock stereo call's two copies take 6.8 ms together, their
 * sum), but a kernel's stores into pinned host memory do run beside a copy
 * engine's H2D (256 MB of kernel stores beside 132 MB of H2D: 4.95 ms;
 * profiles/r06_zc_duplex.json).  So such a call runs in slabs of
 * DUPLEX_SLAB PCM bytes:
 *
 *   g->s_dec       H2D of slab k's XA from the caller's buffer, registered
 *                  for the call (copy engine), then decode slab k (K1 +
 *                  tail); its entry state is read on the device from slab
 *                  k-1's status words
 *   g->s_out       a copy kernel stores slab k's PCM straight into the
 *                  caller's dst when that could be registered (direct), or
 *                  into a pinned staging slot, and its status into the
 *                  slot's header, on CUs of its own (its stores wait on PCIe
 *                  and would hold up a decode sharing their CUs)
 *   calling thread and the copy pool: slot -> the caller's dst (staging)
 *
 * A slot is reused once the host is done with it.  A slab whose status
 * reports a failing block ends the output at that eblock, as the serial
 * route does; nothing is written to dst past it.  BJXA_DUPLEX=0 (read at
 * the first call) keeps every call on the serial route.
 */
#ifndef DUPLEX_SLAB_MIB
#define DUPLEX_SLAB_MIB		16
#endif
#define DUPLEX_SLAB		((size_t)DUPLEX_SLAB_MIB << 20)	/* PCM bytes per slab */
#ifndef DUPLEX_SLOTS
#define DUPLEX_SLOTS		4
#endif
#define DUPLEX_HDR		4096			/* status, then the slab */
#define DUPLEX_MIN_SLABS	(64 / DUPLEX_SLAB_MIB)	/* calls of >= 64 MiB of PCM */
#define DUPLEX_OUT_CUS		64	/* the copy-out stream's CUs; 2 workgroups each */

/*
 * Slab copy-out, HBM -> pinned host memory.  On CDNA one counter (vmcnt)
 * covers loads and stores, so waiting for a load also waits for every
 * store issued before it -- here a store across PCIe.  Each thread loads
 * SLAB_OUT_U pieces before it stores any, so a wave waits for its stores'
 * round trip once per SLAB_OUT_U KiB instead of once per KiB.
 */
#define SLAB_OUT_U	8

__global__ __launch_bounds__(256) void
xa_slab_out(const uint4 *src, uint4 *dst, uint64_t n16, const uint32_t *st,
    uint32_t *st_out)
{
	if (blockIdx.x == 0 && threadIdx.x < XA_ST_WORDS)
		st_out[threadIdx.x] = st[threadIdx.x];
	const uint64_t step = (uint64_t)gridDim.x * 256u * SLAB_OUT_U;
	uint64_t i = blockIdx.x * 256ull * SLAB_OUT_U + threadIdx.x;
	for (; i + 256u * (SLAB_OUT_U - 1) < n16; i += step) {
		uint4 v[SLAB_OUT_U];
#pragma unroll
		for (int u = 0; u < SLAB_OUT_U; u++)
			v[u] = src[i + 256u * u];
#pragma unroll
		for (int u = 0; u < SLAB_OUT_U; u++)
			dst[i + 256u * u] = v[u];
	}
	for (int u = 0; u < SLAB_OUT_U; u++)	/* the last, partial tile */
		if (i + 256u * u < n16)
			dst[i + 256u * u] = src[i + 256u * u];
}

/*
 * The direct form of xa_slab_out, for a decode whose output (the caller's
 * buffer) is registered: the slab's PCM goes straight into it, which spares
 * the host copy out of staging (that copy slowed the kernel's PCIe writes
 * by ~15 %, tools/copyout_probe2.hip).  It writes the slab's `nbytes` cut
 * at its first failing block (its status), and nothing if an earlier slab
 * failed: stop_prev is the word the previous slab's copy-out left (NULL for
 * the first slab), stop_cur this slab's, so no PCM past the failing block
 * reaches the caller, as on the serial route.  The status words go to the
 * slot header for the host, as in xa_slab_out.
 */
__global__ __launch_bounds__(256) void
xa_slab_direct(const uint4 *src, uint8_t *dst, uint64_t nbytes,
    const uint32_t *st, uint32_t *st_out, const uint32_t *stop_prev,
    uint32_t *stop_cur, uint32_t ob, uint32_t ch, uint32_t eb_off,
    uint32_t ek)
{
	/* st: the status of the decode holding this slab at eblock eb_off */
	const uint32_t err = st[XA_ST_ERR];
	const uint32_t errb = err / ch;
	const bool failed = err != 0xffffffffu && errb < eb_off + ek;
	const bool stopped = stop_prev != nullptr && *stop_prev != 0u;
	if (blockIdx.x == 0 && threadIdx.x < XA_ST_WORDS)
		st_out[threadIdx.x] = st[threadIdx.x];
	if (blockIdx.x == 0 && threadIdx.x == 0)
		*stop_cur = stopped || failed ? 1u : 0u;
	if (stopped)
		return;
	if (failed)
		nbytes = errb > eb_off ? min(nbytes, (uint64_t)(errb - eb_off) * ob) : 0u;
	const uint64_t n16 = nbytes / 16u;
	uint4 *d = (uint4 *)dst;
	const uint64_t step = (uint64_t)gridDim.x * 256u * SLAB_OUT_U;
	uint64_t i = blockIdx.x * 256ull * SLAB_OUT_U + threadIdx.x;
	for (; i + 256u * (SLAB_OUT_U - 1) < n16; i += step) {
		uint4 v[SLAB_OUT_U];
#pragma unroll
		for (int u = 0; u < SLAB_OUT_U; u++)
			v[u] = src[i + 256u * u];
#pragma unroll
		for (int u = 0; u < SLAB_OUT_U; u++)
			d[i + 256u * u] = v[u];
	}
	for (int u = 0; u < SLAB_OUT_U; u++)	/* the last, partial tile */
		if (i + 256u * u < n16)
			d[i + 256u * u] = src[i + 256u * u];
	if (blockIdx.x == 0 && threadIdx.x == 0)	/* a cut last block */
		for (uint64_t b = n16 * 16u; b < nbytes; b++)
			dst[b] = ((const uint8_t *)src)[b];
}

static bool
duplex_enabled(void)
{
	static std::once_flag once;
	static bool on;
	std::call_once(once, [] {
		const char *e = getenv("BJXA_DUPLEX");
		on = e == NULL || strcmp(e, "0") != 0;
	});
	return on;
}

/*
 * Are the pages of [p, p + len) in memory (32 pages sampled)?  Registering
 * a buffer whose pages were never touched faults every one of them in, one
 * thread, inside the call: a fresh 256 MB output took the direct route to
 * 16.8 ms against 9.7 through staging, whose host copies fault them in on
 * many threads (tools/host_rate.py --fresh, R6-7).  Such a buffer goes
 * through staging.
 */
static bool
resident(const void *p, size_t len)
{
	const uintptr_t pg = 4096, a = (uintptr_t)p & ~(pg - 1);
	const uintptr_t npg = ((uintptr_t)p + len - a + pg - 1) / pg;
	for (uintptr_t i = 0; i < 32; i++) {
		unsigned char v = 0;
		const uintptr_t q = a + (npg * i / 32) * pg;
		if (mincore((void *)q, pg, &v) != 0 || (v & 1u) == 0)
			return false;
	}
	return true;
}

/*
 * Slabs per decode launch, at most (BJXA_DUPLEX_GROUP, read per call).  A
 * kernel storing into host memory slows every kernel that writes HBM ~20x
 * (tools/clog_probe.hip), so a slab decode runs in the gap between two
 * copy-outs, not beside them; fewer, larger decodes leave fewer gaps.
 * In-process A/B, groups growing 1, 2, 3, 4 (R6-7): a cap of 1 / 4 / 6 /
 * 9 / 16 gave 6.15 / 5.66 / 5.70 / 5.69 / 5.70 ms stereo, 5.92 / 5.62 /
 * 5.67 / 5.66 / 5.65 mono.
 */
#ifndef DUPLEX_GROUP
#define DUPLEX_GROUP	4
#endif

static size_t
duplex_group(void)
{
	const char *e = getenv("BJXA_DUPLEX_GROUP");
	const long v = e != NULL ? strtol(e, NULL, 10) : DUPLEX_GROUP;
	return v < 1 ? 1u : v > 16 ? (size_t)16 : (size_t)v;
}

/*
 * Slabs per encode launch, at most (BJXA_DUPLEX_EGROUP, read per call).  The
 * encode's long direction is its input, which runs back to back on the copy
 * engine once the XA goes straight into the caller's buffer; grouping then
 * only lengthens the last group's copy-outs after the input ends (cap 1 / 4
 * / 8 / 16: 5.79 / 5.88 / 6.24 / 6.24 ms stereo, R6-7), so one slab a launch.
 */
#define DUPLEX_EGROUP	1

static size_t
duplex_egroup(void)
{
	const char *e = getenv("BJXA_DUPLEX_EGROUP");
	const long v = e != NULL ? strtol(e, NULL, 10) : DUPLEX_EGROUP;
	return v < 1 ? 1u : v > 16 ? (size_t)16 : (size_t)v;
}

/*
 * Groups of slabs per kernel launch: first[k] = the first slab of k's
 * group.  Slab 0 alone (the first output as early as possible), then groups
 * growing by half up to gm: a group's input (~0.2 ms a slab beside the
 * copy-outs) has to land within the previous group's copy-outs (~0.33 ms a
 * slab).
 */
static void
duplex_groups(std::vector<size_t> &first, size_t gm)
{
	for (size_t k = 0, a = 0, len = 1; k < first.size(); k++) {
		if (k == a + len) {
			a = k;
			len = std::min(std::max(len + 1, 3 * len / 2), gm);
		}
		first[k] = a;
	}
}

/*
 * BJXA_DUPLEX_DIRECT=1: the copy-out kernel stores the output straight into
 * the caller's buffer, registered for the call (read per call).  Opt-in: a
 * randomised soak of the host API, run right after a long device-side one,
 * ended with the card in a faulted state during a direct-route call, and
 * the cause was not found; the default keeps the
 * kernels' stores in runtime-allocated pinned staging and registers only
 * the input, which only the copy engine reads.
 */
static bool
duplex_direct(void)
{
	const char *e = getenv("BJXA_DUPLEX_DIRECT");
	return e != NULL && strcmp(e, "1") == 0;
}

static std::mutex duplex_pool_mu;
static xa_pool::copy_pool *duplex_pool;

/* the copy pool of the duplex route (process-wide, one job at a time) */
static void
duplex_copy(uint8_t *to, const uint8_t *from, size_t len)
{
	std::lock_guard<std::mutex> lk(duplex_pool_mu);
	try {
		if (duplex_pool == NULL)
			duplex_pool = new xa_pool::copy_pool(xa_pool::pool_threads());
		std::vector<xa_pool::piece> p(1, xa_pool::piece{ to, from, len });
		duplex_pool->run(p);
	} catch (...) {
		memcpy(to, from, len);	/* no memory for the pool: copy here */
	}
}

static int
duplex_setup(struct bjxa__gpu *g, size_t nslab)
{
	if (g->s_out == NULL) {
		/*
		 * The copy-out kernel's stores go over PCIe and back up every
		 * CU's memory pipeline they run on, so a decode kernel sharing
		 * those CUs waits for them (the two serialise, R6-7): the
		 * copy-out stream and the duplex decode stream get disjoint CU
		 * masks.
		 */
		int ncu = 0;
		if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount,
		    g->device) != hipSuccess || ncu <= 0)
			ncu = 256;
		if (ncu > 64 * 32)
			ncu = 64 * 32;
		const unsigned oc = DUPLEX_OUT_CUS;
		const uint32_t nw = (uint32_t)(ncu + 31) / 32;
		uint32_t mo[64] = { 0 }, md[64] = { 0 };	/* (no allocation) */
		const unsigned step = oc > 0 && oc < (unsigned)ncu ? ncu / oc : 1u;
		for (int c = 0; c < ncu; c++) {
			const bool out = oc == 0 || (c % step == 0 &&
			    (unsigned)(c / step) < oc);
			(out ? mo : md)[c / 32] |= 1u << (c % 32);
		}
		bool ok = true;
		if (oc == 0 || oc >= (unsigned)ncu) {
			ok = hipStreamCreateWithFlags(&g->s_out,
			    hipStreamNonBlocking) == hipSuccess &&
			    hipStreamCreateWithFlags(&g->s_dec, hipStreamNonBlocking) ==
			    hipSuccess;
		} else {
			if (hipExtStreamCreateWithCUMask(&g->s_out, nw, mo) !=
			    hipSuccess || hipExtStreamCreateWithCUMask(&g->s_dec, nw,
			    md) != hipSuccess) {
				/* no CU masks here: plain streams (slower, R6-7) */
				(void)hipGetLastError();
				if (g->s_out != NULL)
					(void)hipStreamDestroy(g->s_out);
				g->s_out = NULL;
				ok = hipStreamCreateWithFlags(&g->s_out,
				    hipStreamNonBlocking) == hipSuccess &&
				    (g->s_dec != NULL || hipStreamCreateWithFlags(&g->s_dec,
				    hipStreamNonBlocking) == hipSuccess);
			}
		}
		if (!ok) {
			(void)hipGetLastError();
			if (g->s_out != NULL)
				(void)hipStreamDestroy(g->s_out);
			if (g->s_dec != NULL)
				(void)hipStreamDestroy(g->s_dec);
			g->s_out = g->s_dec = NULL;
			return io_fail();
		}
	}
	if (g->h_stage == NULL) {
		if (hipHostMalloc((void **)&g->h_stage, DUPLEX_SLOTS *
		    (DUPLEX_HDR + DUPLEX_SLAB), hipHostMallocDefault) != hipSuccess) {
			g->h_stage = NULL;
			errno = ENOMEM;
			return -1;
		}
		if (hipHostGetDevicePointer((void **)&g->d_stage, g->h_stage, 0) !=
		    hipSuccess) {
			(void)hipHostFree(g->h_stage);
			g->h_stage = NULL;
			return io_fail();
		}
	}
	if (g->sst_cap < nslab) {
		/* per slab its status words, then per slab a stop word; and the
		 * host's copy of the status words */
		(void)hipFree(g->d_sst);
		g->d_sst = NULL;
		if (g->h_hst != NULL)
			(void)hipHostFree(g->h_hst);
		g->h_hst = g->d_hst = NULL;
		g->sst_cap = 0;
		if (hipHostMalloc((void **)&g->h_hst, nslab * XA_ST_WORDS * 4,
		    hipHostMallocDefault) != hipSuccess) {
			g->h_hst = NULL;
			errno = ENOMEM;
			return -1;
		}
		if (hipHostGetDevicePointer((void **)&g->d_hst, g->h_hst, 0) !=
		    hipSuccess) {
			(void)hipHostFree(g->h_hst);
			g->h_hst = NULL;
			return io_fail();
		}
		if (hipMalloc((void **)&g->d_sst, nslab * (XA_ST_WORDS + 1) * 4) !=
		    hipSuccess) {
			g->d_sst = NULL;
			errno = ENOMEM;
			return -1;
		}
		g->sst_cap = nslab;
	}
	return 0;
}

namespace {

/* at least n events in g's pool (created once, kept across calls: ~2n
 * event creations per call cost more than the route's host work) */
int
event_pool(struct bjxa__gpu *g, size_t n)
{
	if (g->evp_n >= n)
		return 0;
	hipEvent_t *p = (hipEvent_t *)realloc(g->evp, n * sizeof *p);
	if (p == NULL) {
		errno = ENOMEM;
		return -1;
	}
	g->evp = p;
	while (g->evp_n < n) {
		if (hipEventCreateWithFlags(&p[g->evp_n], hipEventDisableTiming) !=
		    hipSuccess) {
			(void)hipGetLastError();
			errno = EIO;
			return -1;
		}
		g->evp_n++;
	}
	return 0;
}

/*
 * The duplex route's registrations of caller memory, process-wide.  A call
 * registers its input's pages (and, for a decode written straight into the
 * caller's buffer, its output's) for the call and unregisters them at its
 * end; another call whose buffers share a page with such a range must not
 * transfer to or from it meanwhile (unregistering under its transfers would
 * take the pages from under a transfer that the runtime or a kernel started
 * on pinned memory).  So a range that lies inside a live registration shares
 * it (a user count), and one that overlaps a registration only in part, or
 * one still being made, waits for it to end.  A call takes all its entries
 * at once and waits only while it holds none, so nothing waits in a cycle.
 * Entries never overlap one another.
 */
struct host_reg {
	uintptr_t	a, b;		/* page range */
	unsigned	users;
	bool		pending;	/* hipHostRegister still running */
	bool		ok;		/* registered by us (else: plain copies) */
};

std::mutex reg_mu;
std::condition_variable reg_cv;
std::list<host_reg> regs;

/* one call's hold on the entries covering its ranges (registered, shared
 * or plain); ranges are page-rounded here and merged when they touch */
struct reg_hold {
	std::list<host_reg>::iterator e[2];
	unsigned n = 0;

	reg_hold(const void *p0, size_t n0, const void *p1, size_t n1)
	{
		uintptr_t r[2][2];
		unsigned nr = 0;
		const void *p[2] = { p0, p1 };
		const size_t len[2] = { n0, n1 };
		for (int i = 0; i < 2; i++)
			if (p[i] != NULL && len[i] != 0) {
				r[nr][0] = (uintptr_t)p[i] & ~(uintptr_t)4095;
				r[nr][1] = ((uintptr_t)p[i] + len[i] + 4095) &
				    ~(uintptr_t)4095;
				nr++;
			}
		if (nr == 2 && r[0][0] <= r[1][1] && r[1][0] <= r[0][1]) {
			r[0][0] = std::min(r[0][0], r[1][0]);
			r[0][1] = std::max(r[0][1], r[1][1]);
			nr = 1;
		}
		bool mine[2] = { false, false };
		std::unique_lock<std::mutex> l(reg_mu);
		for (;;) {
			bool wait = false;
			for (unsigned i = 0; i < nr && !wait; i++)
				for (const host_reg &h : regs)
					if (h.a < r[i][1] && r[i][0] < h.b &&
					    (h.pending || r[i][0] < h.a || h.b < r[i][1])) {
						wait = true;
						break;
					}
			if (!wait)
				break;
			reg_cv.wait(l);
		}
		/* (list nodes allocated up front: nothing below throws while an
		 * entry is half made, which would leave others waiting on it) */
		std::list<host_reg> fresh;
		for (unsigned i = 0; i < nr; i++)
			fresh.push_back(host_reg{ r[i][0], r[i][1], 1u, true, false });
		for (unsigned i = 0; i < nr; i++) {
			auto it = regs.begin();
			while (it != regs.end() && !(it->a <= r[i][0] && r[i][1] <= it->b))
				++it;
			if (it != regs.end()) {
				it->users++;
			} else {
				auto f = fresh.begin();
				for (unsigned j = 0; j < i; j++)
					if (!mine[j])
						++f;
				/* (the node for range i: fresh keeps the unused ones in
				 * order, so skip those of earlier shared ranges) */
				it = f;
				regs.splice(regs.end(), fresh, f);
				mine[i] = true;
			}
			e[n++] = it;
		}
		l.unlock();
		bool ok[2] = { false, false };
		for (unsigned i = 0; i < n; i++)
			if (mine[i]) {
				ok[i] = hipHostRegister((void *)e[i]->a, e[i]->b - e[i]->a,
				    hipHostRegisterDefault) == hipSuccess;
				if (!ok[i])	/* (already pinned, say): plain copies */
					(void)hipGetLastError();
			}
		l.lock();
		for (unsigned i = 0; i < n; i++)
			if (mine[i]) {
				e[i]->pending = false;
				e[i]->ok = ok[i];
			}
		reg_cv.notify_all();
	}

	~reg_hold()
	{
		std::lock_guard<std::mutex> l(reg_mu);
		for (unsigned i = 0; i < n; i++) {
			if (--e[i]->users != 0)
				continue;
			if (e[i]->ok)
				(void)hipHostUnregister((void *)e[i]->a);
			regs.erase(e[i]);
		}
		reg_cv.notify_all();
	}

	/* is [p, p + len) inside an entry this call holds that we registered? */
	bool registered(const void *p, size_t len) const
	{
		std::lock_guard<std::mutex> l(reg_mu);
		for (unsigned i = 0; i < n; i++)
			if (e[i]->ok && e[i]->a <= (uintptr_t)p &&
			    (uintptr_t)p + len <= e[i]->b)
				return true;
		return false;
	}
};

}	/* namespace */

/* BJXA_DUPLEX_TRACE=1: per-slab host timestamps on stderr (diagnostic) */
static double
trace_ms(void)
{
	return std::chrono::duration<double, std::milli>(
	    std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool
duplex_trace(void)
{
	static std::once_flag once;
	static bool on;
	std::call_once(once, [] { on = getenv("BJXA_DUPLEX_TRACE") != NULL; });
	return on;
}

/* staging slot of slab k: its device view, or the host's */
static uint8_t *
duplex_slot(const struct bjxa__gpu *g, size_t k, bool device)
{
	return (device ? g->d_stage : g->h_stage) + (k % DUPLEX_SLOTS) *
	    (DUPLEX_HDR + DUPLEX_SLAB);
}

/*
 * One duplex call over n slabs (decode or encode).  Per slab, on the
 * decode stream: its input H2D, then its kernel; on the copy-out stream,
 * once that kernel is done, its copy-out; the host keeps DUPLEX_SLOTS slabs
 * in flight and reaps them in order.  The input shares the decode stream
 * because an H2D on a stream of its own, behind an event the decode waits
 * on, started only as a copy-out kernel ended (kernel + copy traces: the
 * whole route then ran one stage at a time; -3 to -4 % on the call with
 * the input on the decode stream, R6-7).  The caller's input (in_bytes at
 * src) is registered for the call, so that each H2D is a true asynchronous
 * copy at the link rate (from pageable memory the runtime's staged copies
 * of 8 MiB ran at ~22 GB/s); where registration fails (memory already
 * pinned or registered, say) the copies stay pageable.  With `out`
 * (out_bytes), the caller's output is registered too, and where that works
 * *d_direct is its device view, which the copy-out then writes instead of
 * staging; where it cannot be registered, -2 before anything is
 * enqueued.  Calls whose buffers share pages share or wait for each
 * other's registrations (reg_hold).
 *   in_range(k, &off, &len)    slab k's input bytes [off, off + len)
 *   gpu(k, sd, ev_dec)         enqueue slab k's kernel on sd (the decode
 *                              stream, after its input) and record
 *                              ev_dec[k] there; a decode may hold a slab
 *                              back to run it with later slabs in one
 *                              launch, recording every held slab's event
 *                              then; false on failure
 *   copy_out(k, ev, ev_out)    enqueue slab k's copy-out on g->s_out after
 *                              ev (into the device view of its staging
 *                              slot, duplex_slot(), or *d_direct) and
 *                              record ev_out there; false on failure
 *   host(k, slot)              the calling thread's part once slab k's
 *                              copy-out is done: copy it out of its slot
 *                              (staging) or check its status; returns 1
 *                              to go on, 0 to stop early (an error the
 *                              caller reports), -1 on failure
 * Returns 0 or -1/errno; every enqueued operation has finished on return.
 */
template <class InRange, class Gpu, class Out, class Host>
static int
duplex_run_(struct bjxa__gpu *g, size_t n, const uint8_t *src, size_t in_bytes,
    uint8_t *out, size_t out_bytes, uint8_t **d_direct, InRange &&in_range,
    Gpu &&gpu, Out &&copy_out, Host &&host);

/* (the C ABI lets no exception out: allocations may fail before anything
 * is enqueued, and nothing after that throws) */
template <class InRange, class Gpu, class Out, class Host>
static int
duplex_run(struct bjxa__gpu *g, size_t n, const uint8_t *src, size_t in_bytes,
    uint8_t *out, size_t out_bytes, uint8_t **d_direct, InRange &&in_range,
    Gpu &&gpu, Out &&copy_out, Host &&host)
{
	*d_direct = NULL;
	try {
		return duplex_run_(g, n, src, in_bytes, out, out_bytes, d_direct,
		    in_range, gpu, copy_out, host);
	} catch (...) {
		errno = ENOMEM;
		return -1;
	}
}

template <class InRange, class Gpu, class Out, class Host>
static int
duplex_run_(struct bjxa__gpu *g, size_t n, const uint8_t *src, size_t in_bytes,
    uint8_t *out, size_t out_bytes, uint8_t **d_direct, InRange &&in_range,
    Gpu &&gpu, Out &&copy_out, Host &&host)
{
	if (event_pool(g, 2 * n) < 0)	/* kernel done, copy-out done */
		return -1;
	hipEvent_t *ev_dec = g->evp, *ev_out = ev_dec + n;
	const bool tr = duplex_trace();
	std::vector<double> t_in(n, 0.0), t_iss(n, 0.0), t_out(n, 0.0), t_cp(n, 0.0);
	const double t0 = tr ? trace_ms() : 0.0;

	/* (released on return, after the streams are synchronised) */
	reg_hold reg(src, in_bytes, out, out_bytes);
	const double t_reg = tr ? trace_ms() - t0 : 0.0;
	if (out != NULL && reg.registered(out, out_bytes)) {
		if (hipHostGetDevicePointer((void **)d_direct, out, 0) != hipSuccess) {
			(void)hipGetLastError();
			*d_direct = NULL;
		}
	}
	if (out != NULL && *d_direct == NULL)
		return -2;	/* nothing enqueued: the caller goes on without out */
	/* every slab's input and kernel up front, on the decode stream: they
	 * use no staging, and a kernel that runs beside a copy-out crawls but
	 * is done long before its own copy-out is due */
	uint8_t *d_in = (uint8_t *)g->d_in;
	bool ok = true;
	for (size_t k = 0; ok && k < n; k++) {
		size_t off, len;
		in_range(k, &off, &len);
		ok = hipMemcpyAsync(d_in + off, src + off, len, hipMemcpyHostToDevice,
		    g->s_dec) == hipSuccess && gpu(k, g->s_dec, ev_dec);
		if (tr)
			t_in[k] = trace_ms() - t0;
	}
	/* copy-outs in flight: as many as staging slots, or every slab when
	 * the output is written directly (the host then reads only status
	 * words, g->h_hst) */
	auto issue = [&](size_t k) -> bool {
		if (!copy_out(k, ev_dec[k], ev_out[k]))
			return false;
		if (tr)
			t_iss[k] = trace_ms() - t0;
		return true;
	};
	const size_t depth = *d_direct != NULL ? n : (size_t)DUPLEX_SLOTS;
	for (size_t k = 0; ok && k < std::min(n, depth); k++)
		ok = issue(k);
	for (size_t k = 0; ok && k < n; k++) {
		if (hipEventSynchronize(ev_out[k]) != hipSuccess) {
			ok = false;
			break;
		}
		if (tr)
			t_out[k] = trace_ms() - t0;
		const int r = host(k, *d_direct != NULL ?
		    (const uint8_t *)(g->h_hst + k * XA_ST_WORDS) :
		    duplex_slot(g, k, false));
		if (tr)
			t_cp[k] = trace_ms() - t0;
		if (r <= 0) {
			ok = r == 0;
			break;
		}
		if (k + depth < n)
			ok = issue(k + depth);
	}
	/* everything enqueued has to finish before the buffers are reused */
	const bool synced = hipStreamSynchronize(g->s_dec) == hipSuccess &&
	    hipStreamSynchronize(g->s_out) == hipSuccess;
	if (tr) {
		fprintf(stderr, "duplex %zu slabs, registered %.3f ms, done %.3f ms\n",
		    n, t_reg, trace_ms() - t0);
		for (size_t k = 0; k < n; k++)
			fprintf(stderr, "  slab %2zu in %.3f issued %.3f out %.3f copied %.3f\n",
			    k, t_in[k], t_iss[k], t_out[k], t_cp[k]);
	}
	return synced && ok ? 0 : io_fail();
}

static int
duplex_decode(struct bjxa__gpu *g, const uint8_t *src, uint32_t eblocks,
    unsigned bits, unsigned ch, int16_t state[4], uint8_t *dst,
    uint64_t dst_bytes, uint32_t *err_cb)
{
	const size_t ebsz = (size_t)(bits * 4 + 1) * ch, ob = 64u * ch;
	const uint32_t se = (uint32_t)(DUPLEX_SLAB / ob);	/* eblocks per slab */
	const size_t n = (eblocks + (size_t)se - 1) / se;
	/* decode groups (duplex_groups): 1, 2, 3, 4 ... up to gmax slabs */
	const size_t gmax = duplex_group();
	std::vector<size_t> first(n);
	auto plan = [&](size_t gm) { duplex_groups(first, gm); };
	auto last = [&](size_t k) { return k + 1 == n || first[k + 1] != first[k]; };
	if (duplex_setup(g, n) < 0 || call_buffers(g, eblocks,
	    (uint32_t)std::min((uint64_t)eblocks, (uint64_t)gmax * se), bits, ch) < 0)
		return -1;
	/* (a workspace initialised on g->stream, used on g->s_dec) */
	if (hipStreamSynchronize(g->stream) != hipSuccess)
		return io_fail();
	g->ws_stale = true;	/* cleared when the call completes */
	uint32_t err = 0xffffffffu, fin[XA_ST_WORDS] = { 0 };
	auto slab_eb = [&](size_t k) {
		return (uint32_t)std::min((size_t)eblocks - k * se, (size_t)se);
	};
	/* the PCM straight into the caller's buffer where it can be registered,
	 * is 16-B aligned (the copy-out's stores) and is already in memory;
	 * else through staging */
	bool direct = duplex_direct() && ((uintptr_t)dst & 15u) == 0 &&
	    resident(dst, (size_t)dst_bytes);
	uint32_t *stop = g->d_sst + g->sst_cap * XA_ST_WORDS;
	uint8_t *d_dir = NULL;
	int r;
	/* (where the output cannot be registered after all, duplex_run returns
	 * -2 before enqueueing anything, and the call goes through staging) */
again:
	plan(gmax);
	r = duplex_run(g, n, src, (size_t)eblocks * ebsz,
	    direct ? dst : NULL, (size_t)dst_bytes, &d_dir,
	    [&](size_t k, size_t *off, size_t *len) {
		*off = k * se * ebsz;
		*len = slab_eb(k) * ebsz;
	}, [&](size_t k, hipStream_t sd, hipEvent_t *ev_dec) -> bool {
		if (!last(k))
			return true;	/* with the group's last slab */
		const size_t a = first[k];
		const uint32_t e0 = (uint32_t)(a * se);
		const uint32_t eg = (uint32_t)(k * se + slab_eb(k)) - e0;
		bjxa_hip_stream_t s;
		memset(&s, 0, sizeof s);
		s.d_src = (uint8_t *)g->d_in + (size_t)e0 * ebsz;
		s.d_dst = (uint8_t *)g->d_out + (size_t)e0 * ob;
		s.eblocks = eg;
		s.frames = (uint64_t)eg * 32u;
		s.bits = (uint8_t)bits;
		s.channels = (uint8_t)ch;
		memcpy(s.state, state, sizeof s.state);
		/* the group's status sits at its last slab, its entry state at the
		 * previous group's */
		uint32_t *sst = g->d_sst + k * XA_ST_WORDS;
		if (decode_async(&s, g->d_ws, g->ws_cap, sst, NULL, sd,
		    a > 0 ? g->d_sst + (a - 1) * XA_ST_WORDS : NULL) < 0)
			return false;
		for (size_t j = a; j <= k; j++)
			if (hipEventRecord(ev_dec[j], sd) != hipSuccess)
				return false;
		return true;
	}, [&](size_t j, hipEvent_t ev_done, hipEvent_t ev_o) -> bool {
		/* slab j's copy-out; the status words are its decode group's,
		 * which sit at the group's last slab */
		const size_t a = first[j];
		size_t k = j;
		while (!last(k))
			k++;
		uint32_t *sst = g->d_sst + k * XA_ST_WORDS;
		if (hipStreamWaitEvent(g->s_out, ev_done, 0) != hipSuccess)
			return false;
		{
			const uint32_t ej = slab_eb(j);
			const uint8_t *pj = (const uint8_t *)g->d_out + j * se * ob;
			uint8_t *slot = duplex_slot(g, j, true);
			if (d_dir != NULL) {
				const size_t lo = j * se * ob;
				const size_t hi = std::min((size_t)dst_bytes,
				    lo + (size_t)ej * ob);
				hipLaunchKernelGGL(xa_slab_direct, dim3(2 * DUPLEX_OUT_CUS),
				    dim3(256), 0, g->s_out, (const uint4 *)pj, d_dir + lo,
				    (uint64_t)(hi > lo ? hi - lo : 0), sst,
				    g->d_hst + j * XA_ST_WORDS,
				    j > 0 ? stop + j - 1 : (const uint32_t *)NULL, stop + j,
				    (uint32_t)ob, (uint32_t)ch, (uint32_t)((j - a) * se), ej);
			} else {
				hipLaunchKernelGGL(xa_slab_out, dim3(2 * DUPLEX_OUT_CUS),
				    dim3(256), 0, g->s_out, (const uint4 *)pj,
				    (uint4 *)(slot + DUPLEX_HDR), (uint64_t)ej * ob / 16u, sst,
				    (uint32_t *)slot);
			}
			if (hipGetLastError() != hipSuccess ||
			    hipEventRecord(ev_o, g->s_out) != hipSuccess)
				return false;
		}
		return true;
	}, [&](size_t k, const uint8_t *slot) -> int {
		uint32_t st[XA_ST_WORDS];
		memcpy(st, (const void *)slot, sizeof st);
		/* the status is its decode group's: a failing block in this slab
		 * stops here, one in a later slab of the group later */
		const size_t a = first[k];
		const bool failed = st[XA_ST_ERR] != 0xffffffffu &&
		    a * se + st[XA_ST_ERR] / ch < k * se + slab_eb(k);
		if (failed)
			err = (uint32_t)(a * se * ch) + st[XA_ST_ERR];
		if (d_dir == NULL) {
			const size_t lo = k * se * ob;
			size_t hi = std::min((size_t)dst_bytes, (k * se + slab_eb(k)) * ob);
			if (failed)
				hi = std::min(hi, (size_t)(err / ch) * ob);
			if (hi > lo)
				duplex_copy(dst + lo, slot + DUPLEX_HDR, hi - lo);
		}	/* (direct: the copy-out kernel wrote the PCM, and cut it) */
		if (failed)
			return 0;
		if (last(k))
			memcpy(fin, st, sizeof fin);
		return 1;
	});
	if (r == -2 && direct) {
		direct = false;
		goto again;
	}
	if (r < 0)
		return -1;
	g->ws_stale = false;
	*err_cb = err;
	if (err != 0xffffffffu)
		return err_state(g, err / ch, err % ch, ch, state);
	exit_state(fin, state);
	return 0;
}

/*
 * The same route for a large encode: PCM slabs in on the copy engine (the
 * long direction, 256 MB for a 2M-eblock stereo call), the encode kernel
 * per slab, and its XA (132 MB) streamed by the copy kernel straight into
 * the caller's buffer when it can be registered (every slab in flight, the
 * input back to back), else into pinned staging.  Slabs are independent
 * (the encoder keeps no state, :665-691).
 */
static int
duplex_encode(struct bjxa__gpu *g, const uint8_t *src, uint64_t frames,
    unsigned bits, unsigned ch, uint8_t *dst)
{
	const size_t ebsz = (size_t)(bits * 4 + 1) * ch, ib = 64u * ch;
	const uint32_t eblocks = (uint32_t)((frames + 31) / 32);
	const uint32_t se = (uint32_t)(DUPLEX_SLAB / ib);	/* eblocks per slab */
	const size_t n = (eblocks + (size_t)se - 1) / se;
	const size_t in_bytes = (size_t)frames * 2u * ch;
	if (duplex_setup(g, n) < 0 ||
	    grow(&g->d_in, &g->in_cap, (size_t)eblocks * ib + 256) < 0 ||
	    grow(&g->d_out, &g->out_cap, (size_t)eblocks * ebsz + 256) < 0)
		return -1;
	auto slab_frames = [&](size_t k) {
		return std::min((uint64_t)frames - (uint64_t)k * se * 32u,
		    (uint64_t)se * 32u);
	};
	/* encode groups, as the decode's (through staging: bounded by the
	 * staging slots) */
	const size_t xa_bytes = (size_t)eblocks * ebsz;
	bool direct = duplex_direct() && ((uintptr_t)dst & 15u) == 0 &&
	    resident(dst, xa_bytes);
	std::vector<size_t> first(n);
	auto last = [&](size_t k) { return k + 1 == n || first[k + 1] != first[k]; };
	uint8_t *d_dir = NULL;
	uint32_t *stop = g->d_sst + g->sst_cap * XA_ST_WORDS;
	/* (the direct copy-out reads a status: one that reports no failure) */
	if (direct && hipMemsetAsync(g->d_sst, 0xff, XA_ST_WORDS * 4, g->s_dec) !=
	    hipSuccess)
		return io_fail();
	int r;
again:
	duplex_groups(first, duplex_egroup());
	r = duplex_run(g, n, src, in_bytes, direct ? dst : NULL, xa_bytes, &d_dir,
	    [&](size_t k, size_t *off, size_t *len) {
		*off = k * se * ib;
		*len = (size_t)slab_frames(k) * 2u * ch;
	}, [&](size_t k, hipStream_t sd, hipEvent_t *ev_dec) -> bool {
		if (!last(k))
			return true;	/* with the group's last slab */
		const size_t a = first[k];
		uint64_t fg = 0;
		for (size_t j = a; j <= k; j++)
			fg += slab_frames(j);
		if (bjxa_hip_encode_async((uint8_t *)g->d_in + a * se * ib, fg, bits,
		    ch, (uint8_t *)g->d_out + a * se * ebsz, sd) < 0)
			return false;
		for (size_t j = a; j <= k; j++)
			if (hipEventRecord(ev_dec[j], sd) != hipSuccess)
				return false;
		return true;
	}, [&](size_t j, hipEvent_t ev_done, hipEvent_t ev_o) -> bool {
		if (hipStreamWaitEvent(g->s_out, ev_done, 0) != hipSuccess)
			return false;
		{
			uint8_t *slot = duplex_slot(g, j, true);
			const size_t xk = (size_t)((slab_frames(j) + 31) / 32) * ebsz;
			const uint4 *pj = (const uint4 *)((uint8_t *)g->d_out +
			    j * se * ebsz);
			if (d_dir != NULL) {
				/* exact bytes into the caller's buffer */
				hipLaunchKernelGGL(xa_slab_direct, dim3(2 * DUPLEX_OUT_CUS),
				    dim3(256), 0, g->s_out, pj, d_dir + j * se * ebsz,
				    (uint64_t)xk, (const uint32_t *)g->d_sst,
				    g->d_hst + j * XA_ST_WORDS,
				    j > 0 ? stop + j - 1 : (const uint32_t *)NULL, stop + j,
				    (uint32_t)ebsz, (uint32_t)ch, 0u, 1u);
			} else {
				/* whole 16-B pieces (the slot has room past the
				 * slab's XA) */
				hipLaunchKernelGGL(xa_slab_out, dim3(2 * DUPLEX_OUT_CUS),
				    dim3(256), 0, g->s_out, pj,
				    (uint4 *)(slot + DUPLEX_HDR), (uint64_t)((xk + 15) / 16),
				    g->d_sst, (uint32_t *)slot);
			}
			if (hipGetLastError() != hipSuccess ||
			    hipEventRecord(ev_o, g->s_out) != hipSuccess)
				return false;
		}
		return true;
	}, [&](size_t k, const uint8_t *slot) -> int {
		if (d_dir != NULL)
			return 1;	/* (the copy-out kernel wrote the XA) */
		const size_t xk = (size_t)((slab_frames(k) + 31) / 32) * ebsz;
		duplex_copy(dst + k * se * ebsz, slot + DUPLEX_HDR, xk);
		return 1;
	});
	if (r == -2 && direct) {
		direct = false;
		goto again;
	}
	return r;
}

extern "C" int
bjxa__gpu_decode(struct bjxa__gpu *g, const void *src, uint32_t eblocks,
    unsigned bits, unsigned ch, int16_t state[4], void *dst,
    uint64_t dst_bytes, uint32_t *err_cb)
{
	device_scope on(g->device);
	if (eblocks <= XA_SMALL_MAX)
		return small_decode(g, src, eblocks, bits, ch, state, dst,
		    dst_bytes, err_cb);
	if (duplex_enabled() && (uint64_t)eblocks * 64u * ch >=
	    DUPLEX_MIN_SLABS * DUPLEX_SLAB) {
		const double t0 = duplex_trace() ? trace_ms() : 0.0;
		const int r = duplex_decode(g, (const uint8_t *)src, eblocks, bits,
		    ch, state, (uint8_t *)dst, dst_bytes, err_cb);
		if (duplex_trace())
			fprintf(stderr, "duplex decode call %.3f ms\n", trace_ms() - t0);
		return r;
	}

	const size_t in_bytes = (size_t)(bits * 4 + 1) * ch * eblocks;
	bjxa_hip_stream_t s;
	uint32_t st[BJXA_HIP_STATUS_WORDS];
	if (call_buffers(g, eblocks, eblocks, bits, ch) < 0)
		return -1;
	/* cleared once the status of this call has come back */
	g->ws_stale = true;
	if (hipMemcpyAsync(g->d_in, src, in_bytes, hipMemcpyHostToDevice,
	    g->stream) != hipSuccess)
		return io_fail();
	s.d_src = g->d_in;
	s.d_dst = g->d_out;
	s.eblocks = eblocks;
	s.frames = (uint64_t)eblocks * 32u;	/* full blocks on the device */
	s.bits = (uint8_t)bits;
	s.channels = (uint8_t)ch;
	memcpy(s.state, state, sizeof s.state);
	if (bjxa_hip_decode_async(&s, g->d_ws, g->ws_cap, g->d_status, NULL,
	    g->stream) < 0)
		return -1;
	if (hipMemcpyAsync(st, g->d_status, sizeof st, hipMemcpyDeviceToHost,
	    g->stream) != hipSuccess || hipStreamSynchronize(g->stream) !=
	    hipSuccess)
		return io_fail();
	g->ws_stale = false;
	*err_cb = st[XA_ST_ERR];
	if (st[XA_ST_ERR] != 0xffffffffu) {
		const uint32_t j = st[XA_ST_ERR] / ch, bad_c = st[XA_ST_ERR] % ch;
		if (dst_bytes > (size_t)j * 64u * ch)
			dst_bytes = (size_t)j * 64u * ch;
		if (err_state(g, j, bad_c, ch, state) < 0)
			return -1;
	} else {
		exit_state(st, state);
	}
	if (dst_bytes > 0 && hipMemcpy(dst, g->d_out, dst_bytes,
	    hipMemcpyDeviceToHost) != hipSuccess)
		return io_fail();
	return 0;
}

extern "C" int
bjxa__gpu_encode(struct bjxa__gpu *g, const void *src, uint64_t frames,
    unsigned bits, unsigned ch, void *dst)
{
	const size_t in_bytes = (size_t)frames * 2u * ch;
	const uint32_t eblocks = (uint32_t)((frames + 31) / 32);
	const size_t out_bytes = (size_t)eblocks * (bits * 4 + 1) * ch;
	device_scope on(g->device);

	if (eblocks <= XA_SMALL_MAX) {
		/* one launch over the pinned buffer */
		if (small_buffer(g) < 0)
			return -1;
		memcpy(g->h_small, src, in_bytes);
		if (xa_small_encode_launch(g->d_small, g->d_small + XA_SMALL_IN,
		    frames, bits, ch, g->stream) != hipSuccess ||
		    hipStreamSynchronize(g->stream) != hipSuccess)
			return io_fail();
		memcpy(dst, g->h_small + XA_SMALL_IN, out_bytes);
		return 0;
	}

	if (duplex_enabled() && (uint64_t)eblocks * 64u * ch >=
	    DUPLEX_MIN_SLABS * DUPLEX_SLAB)
		return duplex_encode(g, (const uint8_t *)src, frames, bits, ch,
		    (uint8_t *)dst);
	if (grow(&g->d_in, &g->in_cap, in_bytes + 256) < 0 ||
	    grow(&g->d_out, &g->out_cap, out_bytes + 256) < 0)
		return -1;
	if (hipMemcpyAsync(g->d_in, src, in_bytes, hipMemcpyHostToDevice,
	    g->stream) != hipSuccess)
		return io_fail();
	if (bjxa_hip_encode_async(g->d_in, frames, bits, ch, g->d_out,
	    g->stream) < 0)
		return -1;
	if (hipMemcpyAsync(dst, g->d_out, out_bytes, hipMemcpyDeviceToHost,
	    g->stream) != hipSuccess || hipStreamSynchronize(g->stream) !=
	    hipSuccess)
		return io_fail();
	return 0;
}

