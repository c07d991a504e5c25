/*
 * xa_decode.hip -- gfx950 XA ADPCM decode: speculative chunked decode with
 * exact verification and repair.
 *
 * Replaces the scalar block loop bjxa_decode (reference src/libbjxa.c:602-661)
 * -> bjxa_inflate_{4,6,8}bits (:286-345) -> bjxa_decode_inflated (:533-578).
 *
 * The predictor state (prev[0], prev[1]) of a channel is carried across every
 * block (:552-571) through a truncating divide and an int16 clamp, so there
 * is no exact associative scan.  The stream is cut into chunks of C eblocks;
 * one lane decodes one chunk (both channels of a stereo chunk: two
 * independent chains per lane):
 *
 *  K1 xa_decode_spec  each lane warms up over the W eblocks before its chunk
 *                     starting from state (0,0) -- exact if a gain-0 block
 *                     occurs there, and two trajectories that meet stay
 *                     together -- then decodes its chunk, emitting PCM.  It
 *                     records g[q] (state it entered the chunk with) and e[q]
 *                     (state it left with).  Chunk 0 starts from the true
 *                     caller state and needs no warm-up.
 *  K2 xa_decode_fix   chunk q is correct iff chunk q-1 is and g[q] == e[q-1].
 *                     Each mismatching chunk re-decodes from e[q-1] block by
 *                     block until its block-end state meets the stored
 *                     trajectory (everything after is then unchanged).  A
 *                     chunk that never meets it rewrites e[q] and queues q+1.
 *  K3 xa_decode_tail  one thread drains that queue in chunk order, so a
 *                     cascade through several chunks is repaired exactly.
 *
 * By induction from chunk 0 every chunk ends up decoded from its true start
 * state: the output is bit-exact for any input, speculation only sets the
 * cost.
 *
 * Memory: each lane's input is contiguous, so lanes read their own 4-block
 * groups with dwordx4 loads (4-byte aligned: a group is 4*(bits*4+1) bytes).
 * Output is staged per wave in LDS (one 64*ch-byte line per lane, padded by
 * 16 B) and written back with each store instruction covering whole lines
 * (128-B lines for stereo, 64-B half lines for mono), instead of 64 lanes
 * each touching a different line.
 */
#include "xa_common.h"
#include "xa_decode.h"

/* ------------------------------------------------------------------ */

__device__ __forceinline__ void
wave_lds_sync()
{
	/* LDS ops of one wave complete in order; stop the compiler moving
	 * them across this point */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(16)));

/* Load one 4-block group (GDW dwords) starting at eblock bg. */
template <int BITS, int CH>
__device__ __forceinline__ void
load_group(uint32_t *w, const uint8_t *src, int64_t bg, uint32_t eblocks)
{
	constexpr int BSZ = BITS * 4 + 1, EBSZ = BSZ * CH, G = 4 / CH;
	constexpr int GDW = BSZ;
	if (bg >= 0 && bg + G <= (int64_t)eblocks) {
		const u32x4 *p = (const u32x4 *)(src + (size_t)bg * EBSZ);
#pragma unroll
		for (int i = 0; i < GDW / 4; i++) {
			u32x4 v = p[i];
			w[4 * i + 0] = v.x;
			w[4 * i + 1] = v.y;
			w[4 * i + 2] = v.z;
			w[4 * i + 3] = v.w;
		}
#pragma unroll
		for (int i = (GDW / 4) * 4; i < GDW; i++)
			w[i] = ((const uint32_t *)p)[i];
	} else {
		/* stream head/tail: guard every dword (the dword holding the
		 * last byte is read whole) */
		const int64_t first = bg * EBSZ / 4;
		const int64_t ndw = ((int64_t)eblocks * EBSZ + 3) / 4;
		const uint32_t *p = (const uint32_t *)src;
#pragma unroll
		for (int i = 0; i < GDW; i++) {
			int64_t d = first + i;
			w[i] = (d >= 0 && d < ndw) ? p[d] : 0u;
		}
	}
}

/*
 * Decode the channel blocks of eblock U of the group held in w, advancing
 * the lane's state and writing the 64*CH output bytes to its LDS line.
 */
template <int BITS, int CH>
__device__ __forceinline__ void
decode_eblock(const uint32_t *w, const int U, int32_t *p0, int32_t *p1,
    uint8_t *line, uint32_t *bad)
{
	constexpr int BSZ = BITS * 4 + 1;
	uint32_t sh[CH];
	int32_t k0[CH], k1[CH];
	*bad = 0;
#pragma unroll
	for (int c = 0; c < CH; c++) {
		uint32_t prof = (w[((U * CH + c) * BSZ) >> 2] >>
		    (8 * (((U * CH + c) * BSZ) & 3))) & 0xffu;
		uint32_t gain = prof >> 4;
		sh[c] = 16u + (prof & 15u);
		xa_gain(gain, k0[c], k1[c]);
		*bad |= (gain >= 5u) ? (1u << c) : 0u;
	}
	if (CH == 2) {
#pragma unroll
		for (int q = 0; q < 8; q++) {
			uint32_t fr[4];
#pragma unroll
			for (int j = 0; j < 4; j++) {
				const int n = 4 * q + j;
				int32_t sl, sr;
				sl = xa_step(code_at<BITS>(w, U * 2 * BSZ, n), sh[0],
				    k0[0], k1[0], p0[0], p1[0]);
				sr = xa_step(code_at<BITS>(w, (U * 2 + 1) * BSZ, n),
				    sh[CH - 1], k0[CH - 1], k1[CH - 1], p0[CH - 1],
				    p1[CH - 1]);
				fr[j] = __builtin_amdgcn_perm((uint32_t)sr,
				    (uint32_t)sl, 0x05040100u);
			}
			u32x4a v = { fr[0], fr[1], fr[2], fr[3] };
			*(u32x4a *)(line + 16 * q) = v;
		}
	} else {
#pragma unroll
		for (int q = 0; q < 4; q++) {
			uint32_t fr[4];
#pragma unroll
			for (int j = 0; j < 4; j++) {
				const int n = 8 * q + 2 * j;
				int32_t a = xa_step(code_at<BITS>(w, U * BSZ, n),
				    sh[0], k0[0], k1[0], p0[0], p1[0]);
				int32_t b = xa_step(code_at<BITS>(w, U * BSZ, n + 1),
				    sh[0], k0[0], k1[0], p0[0], p1[0]);
				fr[j] = __builtin_amdgcn_perm((uint32_t)b,
				    (uint32_t)a, 0x05040100u);
			}
			u32x4a v = { fr[0], fr[1], fr[2], fr[3] };
			*(u32x4a *)(line + 16 * q) = v;
		}
	}
}

/*
 * K1.  One lane per chunk.  Block geometry is fully compile-time inside a
 * group; the loop over groups is the only runtime loop.
 */
template <int BITS, int CH>
__global__ __launch_bounds__(256) void
xa_decode_spec(xa_dec_args a)
{
	constexpr int G = 4 / CH;
	constexpr int GDW = BITS * 4 + 1;
	constexpr int OB = 64 * CH;		/* output bytes per eblock */
	constexpr int LINE = OB + 16;		/* padded LDS line */
	constexpr int PIECES = OB / 16;		/* 16-B pieces per line */
	__shared__ __attribute__((aligned(16))) uint8_t stage[4 * 64 * LINE];

	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	uint8_t *wbase = stage + wv * 64 * LINE;
	uint8_t *line = wbase + lane * LINE;
	const uint32_t chunk = blockIdx.x * 256u + threadIdx.x;
	const uint32_t wchunk0 = blockIdx.x * 256u + wv * 64u;
	const int64_t b0 = (int64_t)chunk * a.C;
	const int64_t start = b0 - (int64_t)a.W;

	int32_t p0[CH], p1[CH];
#pragma unroll
	for (int c = 0; c < CH; c++) {
		if (start < 0)
			xa_unpack_state(a.init[c], p0[c], p1[c]);
		else
			p0[c] = p1[c] = 0;
	}
	uint32_t gst[CH];
#pragma unroll
	for (int c = 0; c < CH; c++)
		gst[c] = 0;

	const int ngroups = (int)((a.W + a.C) / G);
	uint32_t w[GDW], wn[GDW];
	load_group<BITS, CH>(w, a.src, start, a.eblocks);

	for (int gi = 0; gi < ngroups; gi++) {
		const int64_t bg = start + (int64_t)gi * G;
		if (gi + 1 < ngroups)
			load_group<BITS, CH>(wn, a.src, bg + G, a.eblocks);
#pragma unroll
		for (int u = 0; u < G; u++) {
			const int64_t b = bg + u;
			const bool act = b >= 0 && b < (int64_t)a.eblocks;
			if (b == b0) {
#pragma unroll
				for (int c = 0; c < CH; c++)
					gst[c] = xa_pack_state(p0[c], p1[c]);
			}
			if (act) {
				uint32_t bad;
				decode_eblock<BITS, CH>(w, u, p0, p1, line, &bad);
				if (bad && b >= b0) {
					uint32_t cb = (uint32_t)b * CH + ((bad & 1u) ? 0u : 1u);
					atomicMin(&a.ctl[XA_CTL_ERR], cb);
				}
			}
			/* wave-uniform: s is the same block offset for every lane */
			const int s = gi * G + u - (int)a.W;
			if (s >= 0) {
				wave_lds_sync();
#pragma unroll
				for (int i = 0; i < PIECES; i++) {
					const int P = i * 64 + lane;
					const int j = P / PIECES, pc = P % PIECES;
					const uint32_t cj = wchunk0 + (uint32_t)j;
					const uint64_t bj = (uint64_t)cj * a.C + (uint64_t)s;
					if (cj < a.nchunks && bj < a.eblocks) {
						const uint64_t off = bj * OB + (uint64_t)pc * 16u;
						const uint8_t *from = wbase + j * LINE + pc * 16;
						if (off + 16u <= a.pcm_bytes) {
							*(u32x4a *)(a.dst + off) = *(const u32x4a *)from;
						} else if (off < a.pcm_bytes) {
							for (uint64_t k = 0; off + k < a.pcm_bytes; k += 2)
								*(uint16_t *)(a.dst + off + k) =
								    *(const uint16_t *)(from + k);
						}
					}
				}
				wave_lds_sync();
			}
		}
#pragma unroll
		for (int i = 0; i < GDW; i++)
			w[i] = wn[i];
	}
	if (chunk < a.nchunks) {
		uint2 gv, ev;
		gv.x = gst[0];
		gv.y = gst[CH - 1];
		ev.x = xa_pack_state(p0[0], p1[0]);
		ev.y = xa_pack_state(p0[CH - 1], p1[CH - 1]);
		if (CH == 1) {
			gv.y = 0;
			ev.y = 0;
		}
		a.g[chunk] = gv;
		a.e[chunk] = ev;
	}
}

/* ------------------------------------------------------------------ */
/* repair path: plain per-thread decode, byte loads, direct stores      */

template <int BITS>
__device__ __forceinline__ int32_t
code_slow(const uint8_t *data, int n)
{
	if (BITS == 8)
		return (int32_t)((uint32_t)data[n] << 24);
	if (BITS == 4) {
		uint32_t v = (uint32_t)data[n >> 1] << 24;
		return (int32_t)((n & 1) ? (v << 4) : (v & 0xf0000000u));
	}
	const int grp = n >> 2, k = n & 3;
	uint32_t g24 = ((uint32_t)data[3 * grp] << 16) |
	    ((uint32_t)data[3 * grp + 1] << 8) | data[3 * grp + 2];
	return (int32_t)(((g24 >> (18 - 6 * k)) & 63u) << 26);
}

/*
 * Re-decode chunk q from state `s`, rewriting its PCM.  Stops early once a
 * block-end state equals the stored trajectory's (then nothing after it can
 * change).  Returns true if it met the stored trajectory; otherwise stores
 * the new end state in e[q].
 */
template <int BITS, int CH>
__device__ bool
fix_chunk(const xa_dec_args &a, uint32_t q, uint2 s)
{
	constexpr int BSZ = BITS * 4 + 1, EBSZ = BSZ * CH, OB = 64 * CH;
	int32_t p0[CH], p1[CH];
	xa_unpack_state(s.x, p0[0], p1[0]);
	if (CH == 2)
		xa_unpack_state(s.y, p0[CH - 1], p1[CH - 1]);
	const uint64_t b0 = (uint64_t)q * a.C;
	uint64_t b1 = b0 + a.C;
	if (b1 > a.eblocks)
		b1 = a.eblocks;
	for (uint64_t b = b0; b < b1; b++) {
		const bool last = b + 1 == a.eblocks;
		uint8_t *out = a.dst + b * OB;
		uint32_t old[CH];
		if (!last) {
			if (CH == 2) {
				uint32_t f31 = *(const uint32_t *)(out + 31 * 4);
				uint32_t f30 = *(const uint32_t *)(out + 30 * 4);
				old[0] = (f31 & 0xffffu) | (f30 << 16);
				old[CH - 1] = (f31 >> 16) | (f30 & 0xffff0000u);
			} else {
				uint32_t f = *(const uint32_t *)(out + 30 * 2);
				old[0] = (f >> 16) | (f << 16);
			}
		}
		for (int c = 0; c < CH; c++) {
			const uint8_t *blk = a.src + b * EBSZ + c * BSZ;
			uint32_t prof = blk[0], gain = prof >> 4;
			uint32_t sh = 16u + (prof & 15u);
			int32_t k0, k1;
			xa_gain(gain, k0, k1);
			for (int n = 0; n < XA_FRAMES; n++) {
				int32_t v = xa_step(code_slow<BITS>(blk + 1, n), sh,
				    k0, k1, p0[c], p1[c]);
				uint64_t off = b * OB + (uint64_t)(n * CH + c) * 2u;
				if (off < a.pcm_bytes)
					*(int16_t *)(a.dst + off) = (int16_t)v;
			}
		}
		if (!last) {
			bool met = true;
			for (int c = 0; c < CH; c++)
				met = met && xa_pack_state(p0[c], p1[c]) == old[c];
			if (met)
				return true;
		}
	}
	uint2 ev;
	ev.x = xa_pack_state(p0[0], p1[0]);
	ev.y = CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u;
	a.e[q] = ev;
	return false;
}

/* K2.  One thread per chunk; only mismatching chunks do work. */
template <int BITS, int CH>
__global__ __launch_bounds__(256) void
xa_decode_fix(xa_dec_args a)
{
	const uint32_t q = blockIdx.x * 256u + threadIdx.x;
	if (q == 0 || q >= a.nchunks)
		return;
	/* e[q-1] may be rewritten concurrently by chunk q-1's fixer; whichever
	 * value is read is recorded in g[q], and that fixer queues q for the
	 * tail pass, which re-checks it */
	const uint2 s = __hip_atomic_load(&a.e[q - 1], __ATOMIC_RELAXED,
	    __HIP_MEMORY_SCOPE_AGENT);
	const uint2 gq = a.g[q];
	if (s.x == gq.x && s.y == gq.y)
		return;
	atomicAdd(&a.ctl[XA_CTL_FIXED], 1u);
	const bool met = fix_chunk<BITS, CH>(a, q, s);
	a.g[q] = s;
	if (!met && q + 1 < a.nchunks) {
		uint32_t i = atomicAdd(&a.ctl[XA_CTL_NQ], 1u);
		a.queue[i] = q + 1;
	}
}

/* K3.  A single thread drains the re-check queue in chunk order. */
template <int BITS, int CH>
__global__ __launch_bounds__(64) void
xa_decode_tail(xa_dec_args a)
{
	if (threadIdx.x != 0)
		return;
	uint32_t n = a.ctl[XA_CTL_NQ], tail = 0;
	while (n > 0) {
		uint32_t mi = 0;
		for (uint32_t i = 1; i < n; i++)
			if (a.queue[i] < a.queue[mi])
				mi = i;
		const uint32_t q = a.queue[mi];
		a.queue[mi] = a.queue[--n];
		const uint2 s = a.e[q - 1], gq = a.g[q];
		if (s.x == gq.x && s.y == gq.y)
			continue;
		tail++;
		const bool met = fix_chunk<BITS, CH>(a, q, s);
		a.g[q] = s;
		if (!met && q + 1 < a.nchunks)
			a.queue[n++] = q + 1;
	}
	const uint2 fin = a.e[a.nchunks - 1];
	a.status[XA_ST_ERR] = a.ctl[XA_CTL_ERR];
	a.status[XA_ST_STATE_L] = fin.x;
	a.status[XA_ST_STATE_R] = fin.y;
	a.status[XA_ST_FIXED] = a.ctl[XA_CTL_FIXED];
	a.status[XA_ST_TAIL] = tail;
	a.status[XA_ST_CHUNKS] = a.nchunks;
	a.ctl[XA_CTL_ERR] = 0xffffffffu;
	a.ctl[XA_CTL_NQ] = 0;
	a.ctl[XA_CTL_FIXED] = 0;
}

/* ------------------------------------------------------------------ */

template <int BITS, int CH>
static hipError_t
launch(const xa_dec_args &a, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1)
{
	const unsigned grid = (a.nchunks + 255u) / 256u;
	if (ev0 != NULL)
		(void)hipEventRecord(ev0, st);
	hipLaunchKernelGGL((xa_decode_spec<BITS, CH>), dim3(grid), dim3(256), 0,
	    st, a);
	if (ev1 != NULL)
		(void)hipEventRecord(ev1, st);
	hipLaunchKernelGGL((xa_decode_fix<BITS, CH>), dim3(grid), dim3(256), 0,
	    st, a);
	hipLaunchKernelGGL((xa_decode_tail<BITS, CH>), dim3(1), dim3(64), 0, st,
	    a);
	return hipGetLastError();
}

hipError_t
xa_decode_launch(const xa_dec_args &a, unsigned bits, unsigned ch,
    hipStream_t st, hipEvent_t ev0, hipEvent_t ev1)
{
	if (ch == 1) {
		if (bits == 8)
			return launch<8, 1>(a, st, ev0, ev1);
		if (bits == 6)
			return launch<6, 1>(a, st, ev0, ev1);
		return launch<4, 1>(a, st, ev0, ev1);
	}
	if (bits == 8)
		return launch<8, 2>(a, st, ev0, ev1);
	if (bits == 6)
		return launch<6, 2>(a, st, ev0, ev1);
	return launch<4, 2>(a, st, ev0, ev1);
}
