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
 *                     The last workgroup to finish (arrival ticket) drains
 *                     that queue in chunk order with one thread, so a
 *                     cascade through several chunks is repaired exactly.
 *
 * By induction from chunk 0 every chunk ends up decoded from its true start
 * state: the output is bit-exact for any input; speculation only sets the
 * cost.
 *
 * Memory (K1).  Loops advance one "group" = 4 channel blocks (2 stereo or 4
 * mono eblocks) = 4*(bits*4+1) bytes, a whole number of dwords.  Each wave
 * owns two LDS regions:
 *  - input: the group of each of its 64 chunks, fetched by LDS-DMA with the
 *    64 segments concatenated so every DMA instruction reads ~256 contiguous
 *    bytes (instead of 64 scattered 16-B pieces, which saturated the texture
 *    addresser).  A lane copies its segment to VGPRs and the next group's
 *    DMA is issued at once, overlapping the decode.
 *  - output: one 64-B line per lane (a mono block, or half a stereo eblock),
 *    written back so each store instruction covers 16 whole 64-B lines.
 *    The DMA wait is a counted vmcnt that leaves those stores in flight.
 */
#include <type_traits>

#include "xa_common.h"
#include "xa_decode.h"

#ifndef XA_SPEC_WPB
#define XA_SPEC_WPB 4		/* waves per workgroup */
#endif
#ifndef XA_DMA_AUX
#define XA_DMA_AUX 0		/* cache policy bits of the input LDS-DMA */
#endif

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

/* compile-time loop: f(integral_constant<int, I>) for I in [I, N) */
template <int I, int N> struct sfor {
	template <typename F>
	__device__ __forceinline__ static void run(F &f)
	{
		f(std::integral_constant<int, I>());
		sfor<I + 1, N>::run(f);
	}
};
template <int N> struct sfor<N, N> {
	template <typename F>
	__device__ __forceinline__ static void run(F &) {}
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(16)));
#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

/* block geometry, all compile-time */
template <int BITS, int CH> struct geo {
	static constexpr int BSZ = BITS * 4 + 1;	/* channel block */
	static constexpr int EBSZ = BSZ * CH;		/* effective block */
	static constexpr int G = 4 / CH;		/* eblocks per group */
	static constexpr int GDW = BSZ;			/* dwords per group */
	static constexpr int OB = 64 * CH;		/* PCM bytes per eblock */
	/* window of eblock u (0..G-1) of a group: first dword, byte offset */
	static constexpr int wbase(int u) { return (u * EBSZ) >> 2; }
	static constexpr int woff(int u) { return (u * EBSZ) & 3; }
	static constexpr int wlen(int u) { return (woff(u) + EBSZ + 3) >> 2; }
	static constexpr int wmax() {
		int m = 0;
		for (int u = 0; u < G; u++)
			m = wlen(u) > m ? wlen(u) : m;
		return m;
	}
	static constexpr int WD = wmax();
};

/*
 * Load the window of eblock b (b % G == U) into w (repair path).  Whole
 * dwords only; the dword holding the stream's last byte is read whole,
 * nothing past it.
 */
template <int BITS, int CH, int U>
__device__ __forceinline__ void
load_window(uint32_t *w, const uint8_t *src, int64_t b)
{
	typedef geo<BITS, CH> g;
	constexpr int N = g::wlen(U);
	const uint32_t *p = (const uint32_t *)(src + (size_t)(b - U) * g::EBSZ) +
	    g::wbase(U);
#pragma unroll
	for (int i = 0; i < N / 4; i++) {
		u32x4 v = ((const u32x4 *)p)[i];
		w[4 * i + 0] = v.x;
		w[4 * i + 1] = v.y;
		w[4 * i + 2] = v.z;
		w[4 * i + 3] = v.w;
	}
#pragma unroll
	for (int i = (N / 4) * 4; i < N; i++)
		w[i] = p[i];
}

/* load_window with every dword index clamped into the stream (no branch) */
template <int BITS, int CH, int U>
__device__ __forceinline__ void
load_window_clamped(uint32_t *w, const uint8_t *src, int64_t b, int64_t ndw)
{
	typedef geo<BITS, CH> g;
	constexpr int N = g::wlen(U);
	const int64_t d0 = (b - U) * g::EBSZ / 4 + g::wbase(U);
	const uint32_t *p = (const uint32_t *)src;
#pragma unroll
	for (int i = 0; i < N; i++)
		w[i] = p[min(d0 + i, ndw - 1)];
}

/*
 * Decode the channel blocks of one eblock whose first byte is byte O of w,
 * advancing the lane's state.  With STORE the output goes to `line` in
 * 16-B pieces; after every LB bytes `flush(h)` runs (h = LB-byte line
 * index), and with RESTART the next line is written at `line` again (LDS
 * staging), otherwise output continues at line + LB (direct stores).
 * Returns a bit per channel whose gain nibble is >= 5.
 */
template <int BITS, int CH, bool STORE, bool RESTART, int LB, typename F>
__device__ __forceinline__ uint32_t
decode_eblock(const uint32_t *w, const int O, int32_t *p0, int32_t *p1,
    uint8_t *line, F &flush)
{
	constexpr int BSZ = BITS * 4 + 1;
	uint32_t sh[CH], bad = 0;
	int32_t k0[CH], k1[CH];
#pragma unroll
	for (int c = 0; c < CH; c++) {
		const int pb = O + c * BSZ;
		uint32_t prof = (w[pb >> 2] >> (8 * (pb & 3))) & 0xffu;
		uint32_t gain = prof >> 4;
		sh[c] = 16u + (prof & 15u);
		xa_gain(gain & 7u, k0[c], k1[c]);
		bad |= (gain >= 5u) ? (1u << c) : 0u;
	}
	/* 16-B piece q holds 4 stereo frames or 8 mono samples */
#pragma unroll
	for (int q = 0; q < 4 * CH; q++) {
		uint32_t fr[4];
#pragma unroll
		for (int j = 0; j < 4; j++) {
			if (CH == 2) {
				const int n = 4 * q + j;
				int32_t sl = xa_step(code_at<BITS>(w, O, n), sh[0],
				    k0[0], k1[0], p0[0], p1[0]);
				int32_t sr = xa_step(code_at<BITS>(w, O + BSZ, n),
				    sh[CH - 1], k0[CH - 1], k1[CH - 1], p0[CH - 1],
				    p1[CH - 1]);
				fr[j] = __builtin_amdgcn_perm((uint32_t)sr,
				    (uint32_t)sl, 0x05040100u);
			} else {
				const int n = 8 * q + 2 * j;
				int32_t sa = xa_step(code_at<BITS>(w, O, n), sh[0],
				    k0[0], k1[0], p0[0], p1[0]);
				int32_t sb = xa_step(code_at<BITS>(w, O, n + 1), sh[0],
				    k0[0], k1[0], p0[0], p1[0]);
				fr[j] = __builtin_amdgcn_perm((uint32_t)sb,
				    (uint32_t)sa, 0x05040100u);
			}
		}
		if (STORE) {
			u32x4a v = { fr[0], fr[1], fr[2], fr[3] };
			constexpr int QL = LB / 16;	/* pieces per line */
			*(u32x4a *)(line + 16 * (RESTART ? (q % QL) : q)) = v;
			if (q % QL == QL - 1)
				flush(q / QL);
		}
		/* keep the unpack of later codes from being hoisted here: it
		 * would only raise register pressure */
		__builtin_amdgcn_sched_barrier(0);
	}
	return bad;
}

/*
 * Store the wave's staged LB-byte lines: line j belongs to chunk
 * wchunk0 + j and goes to byte `rel_off` of that chunk's PCM.  Lane l
 * stores piece l % P of lines l / P + (64 / P) i (P = LB / 16 pieces per
 * line).  Wave-uniform fast path when every line is whole; otherwise (the
 * grid's last wave only) per-piece bounds and a 2-byte tail for the
 * stream's cut last block.
 */
template <int LB, bool NT>
__device__ __forceinline__ void
store_lines(const xa_dec_args &a, const uint8_t *obuf, int lane,
    uint32_t wchunk0, uint32_t chunk_bytes, uint32_t rel_off, bool wave_full,
    uint8_t *gbase, const uint8_t *lbase)
{
	constexpr int LINE = LB + 16, P = LB / 16, LPI = 64 / P;
	if (wave_full) {
		uint8_t *gp = gbase + rel_off;
		const uint64_t istride = (uint64_t)LPI * chunk_bytes;
#pragma unroll
		for (int i = 0; i < P; i++) {
			const u32x4a v = *(const u32x4a *)(lbase + i * LPI * LINE);
			if (NT)
				__builtin_nontemporal_store(v,
				    (u32x4a *)(gp + i * istride));
			else
				*(u32x4a *)(gp + i * istride) = v;
		}
		return;
	}
	/* launder the inputs so none of this rare path's address arithmetic
	 * is hoisted out of the caller's loops (it would pin ~100 VGPRs) */
	uint32_t wc = wchunk0, nch = a.nchunks, cb = chunk_bytes, ro = rel_off;
	uint64_t lim = a.pcm_bytes;
	uint8_t *dst = a.dst;
	asm volatile("" : "+v"(wc), "+v"(nch), "+v"(cb), "+v"(ro), "+v"(lim),
	    "+v"(dst));
#pragma nounroll
	for (int i = 0; i < P; i++) {
		const int j = i * LPI + lane / P, pc = lane % P;
		const uint32_t cj = wc + (uint32_t)j;
		const uint64_t off = (uint64_t)cj * cb + ro + (uint64_t)pc * 16u;
		if (cj >= nch)
			continue;
		const uint8_t *from = obuf + j * LINE + pc * 16;
		if (off + 16u <= lim) {
			*(u32x4a *)(dst + off) = *(const u32x4a *)from;
		} else if (off < lim) {
			for (uint64_t k = 0; off + k < lim; k += 2)
				*(uint16_t *)(dst + off + k) =
				    *(const uint16_t *)(from + k);
		}
	}
}

/*
 * Stage one group of each of the wave's 64 chunks into `ibuf` by LDS-DMA:
 * the 64 segments are concatenated and instruction i moves dwords
 * [64i, 64i+64) of that concatenation (lane t: dword 64i+t).  `rel` is the
 * group's first eblock relative to each chunk's start.  Segments outside
 * the stream (warm-up before eblock 0, the ragged end) are clamped onto
 * valid dwords; their lanes never decode them.
 */
template <int BITS, int CH>
__device__ __forceinline__ void
stage_group(const xa_dec_args &a, uint8_t *ibuf, int lane, uint32_t wchunk0,
    int64_t rel, const uint32_t *voff)
{
	typedef geo<BITS, CH> g;
	constexpr int GDW = g::GDW;
	const int64_t e_first = (int64_t)wchunk0 * a.C + rel;
	const int64_t e_end = (int64_t)(wchunk0 + 63u) * a.C + rel + g::G;
	if (e_first >= 0 && e_end <= (int64_t)a.eblocks) {
		const uint8_t *base = a.src + (size_t)e_first * g::EBSZ;
#pragma unroll
		for (int i = 0; i < GDW; i++)
			__builtin_amdgcn_global_load_lds(
			    (const void *)(base + voff[i]), LDS_PTR(ibuf + i * 256),
			    4, 0, XA_DMA_AUX);
		return;
	}
	/* rare path (the grid's first and last waves): launder the inputs so
	 * none of its arithmetic is hoisted into the caller's loops */
	uint32_t wc = wchunk0, C = a.C, neb = a.eblocks;
	int64_t r = rel;
	const uint8_t *src = a.src;
	asm volatile("" : "+v"(wc), "+v"(C), "+v"(neb), "+v"(r), "+v"(src));
	const int64_t last = ((int64_t)neb * g::EBSZ - 1) & ~(int64_t)3;
#pragma nounroll
	for (int i = 0; i < GDW; i++) {
		const int k = i * 64 + lane, seg = k / GDW, off = k % GDW;
		int64_t byte = ((int64_t)(wc + seg) * C + r) * g::EBSZ + off * 4;
		byte = byte < 0 ? 0 : (byte > last ? last : byte);
		__builtin_amdgcn_global_load_lds((const void *)(src + byte),
		    LDS_PTR(ibuf + i * 256), 4, 0, XA_DMA_AUX);
	}
}

/*
 * K1.  One lane per chunk, XA_SPEC_WPB waves per workgroup.
 *  SPLIT  separate input and output LDS regions: the next group's DMA is
 *         issued before the decode and waited for with a counted vmcnt that
 *         leaves the group's stores in flight.  Otherwise one region serves
 *         both and the DMA follows the group's last store phase.
 *  LB     output line bytes per lane per store phase (64, or the eblock's
 *         64*ch).
 */
template <int BITS, int CH, bool SPLIT, int LB, bool NT>
__global__ __launch_bounds__(64 * XA_SPEC_WPB) void
xa_decode_spec(xa_dec_args a)
{
	typedef geo<BITS, CH> g;
	constexpr int G = g::G, OB = g::OB, EBSZ = g::EBSZ, GDW = g::GDW;
	constexpr int IBUF = 64 * GDW * 4;	/* input stage, per wave */
	constexpr int LINE = LB + 16;		/* output line + pad */
	constexpr int OBUF = 64 * LINE;		/* output stage, per wave */
	constexpr int REGION = SPLIT ? IBUF + OBUF : (IBUF > OBUF ? IBUF : OBUF);
	/* stores issued between a group's DMA and the next group's wait */
	constexpr int STORES_PER_GROUP = G * OB / 16;
	__shared__ __attribute__((aligned(16))) uint8_t
	    lds[XA_SPEC_WPB * REGION];

	/* the wave index is wave-uniform; say so, so that LDS bases and the
	 * DMA source base live in SGPRs */
	const int lane = threadIdx.x & 63;
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	uint8_t *ibuf = lds + wv * REGION;
	uint8_t *obuf = SPLIT ? ibuf + IBUF : ibuf;
	uint8_t *line = obuf + lane * LINE;
	const uint32_t wchunk0 = blockIdx.x * (64u * XA_SPEC_WPB) + wv * 64u;
	const uint32_t chunk = wchunk0 + lane;
	const int64_t eblocks = a.eblocks;
	const int64_t b0 = (int64_t)chunk * a.C;
	const int W = (int)a.W;

	/* DMA source offsets (bytes from the wave's segment 0) of this lane's
	 * dword in each stage instruction; the same for every group */
	uint32_t voff[GDW];
#pragma unroll
	for (int i = 0; i < GDW; i++) {
		const int k = i * 64 + lane;
		voff[i] = (uint32_t)(k / GDW) * a.C * EBSZ + (uint32_t)(k % GDW) * 4u;
	}

	int32_t p0[CH], p1[CH];
#pragma unroll
	for (int c = 0; c < CH; c++) {
		if (b0 - W < 0)
			xa_unpack_state(a.init[c], p0[c], p1[c]);
		else
			p0[c] = p1[c] = 0;
	}

	uint32_t w[GDW];
	const uint32_t *mine = (const uint32_t *)(ibuf + lane * GDW * 4);
	auto none = [](int) {};
	stage_group<BITS, CH>(a, ibuf, lane, wchunk0, -W, voff);

	/* warm-up: state only; the next group's DMA overlaps the decode */
	for (int rel = -W; rel < 0; rel += G) {
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
		for (int i = 0; i < GDW; i++)
			w[i] = mine[i];
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		stage_group<BITS, CH>(a, ibuf, lane, wchunk0, rel + G, voff);
		auto body = [&](auto uc) {
			constexpr int u = decltype(uc)::value;
			const int64_t b = b0 + rel + u;
			if (b >= 0 && b < eblocks)
				(void)decode_eblock<BITS, CH, false, true, 64>(w,
				    u * EBSZ, p0, p1, line, none);
		};
		sfor<0, G>::run(body);
	}
	uint32_t gst[2];
	gst[0] = xa_pack_state(p0[0], p1[0]);
	gst[1] = CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u;

	/* the chunk: decode, stage 64-B lines, write them back whole */
	const uint32_t chunk_bytes = a.C * OB;
	constexpr int P = LB / 16;
	uint8_t *gbase = a.dst + (uint64_t)(wchunk0 + lane / P) * chunk_bytes +
	    (lane % P) * 16;
	const uint8_t *lbase = obuf + (lane / P) * LINE + (lane % P) * 16;
	/* every line of this wave lies before the stream's first cut block */
	const uint64_t full_blocks = a.pcm_bytes / OB;
	const bool wave_full = wchunk0 + 63u < a.nchunks &&
	    (uint64_t)(wchunk0 + 64u) * a.C <= full_blocks;
	bool first = true;
	for (int s0 = 0; s0 < (int)a.C; s0 += G) {
		/* this group's DMA, not the previous group's stores */
		if (!SPLIT || first || !wave_full)
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		else
			asm volatile("s_waitcnt vmcnt(%0)" :: "n"(STORES_PER_GROUP)
			    : "memory");
		first = false;
#pragma unroll
		for (int i = 0; i < GDW; i++)
			w[i] = mine[i];
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		if (SPLIT && s0 + G < (int)a.C)
			stage_group<BITS, CH>(a, ibuf, lane, wchunk0, s0 + G, voff);
		auto body = [&](auto uc) {
			constexpr int u = decltype(uc)::value;
			const int s = s0 + u;
			const int64_t b = b0 + s;
			auto flush = [&](int h) {
				wave_lds_sync();
				store_lines<LB, NT>(a, obuf, lane, wchunk0, chunk_bytes,
				    (uint32_t)s * OB + (uint32_t)LB * h, wave_full, gbase,
				    lbase);
				wave_lds_sync();
			};
			/* every lane runs the decode (flush holds wave-wide
			 * stores); past the stream's end -- only in the last
			 * chunk -- it decodes padding and keeps its old state */
			const bool act = b < eblocks;
			int32_t q0[CH], q1[CH];
#pragma unroll
			for (int c = 0; c < CH; c++) {
				q0[c] = p0[c];
				q1[c] = p1[c];
			}
			uint32_t bad = decode_eblock<BITS, CH, true, true, LB>(w,
			    u * EBSZ, p0, p1, line, flush);
			if (act && bad) {
				uint32_t cb = (uint32_t)b * CH + ((bad & 1u) ? 0u : 1u);
				atomicMin(&a.ctl[XA_CTL_ERR], cb);
			}
#pragma unroll
			for (int c = 0; c < CH; c++) {
				p0[c] = act ? p0[c] : q0[c];
				p1[c] = act ? p1[c] : q1[c];
			}
		};
		sfor<0, G>::run(body);
		if (!SPLIT && s0 + G < (int)a.C) {
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			stage_group<BITS, CH>(a, ibuf, lane, wchunk0, s0 + G, voff);
		}
	}
	if (chunk < a.nchunks) {
		uint2 gv, ev;
		gv.x = gst[0];
		gv.y = gst[1];
		ev.x = xa_pack_state(p0[0], p1[0]);
		ev.y = CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u;
		a.g[chunk] = gv;
		a.e[chunk] = ev;
	}
}

/* ------------------------------------------------------------------ */
/* repair path                                                          */

/*
 * Re-decode chunk q from state `s`, rewriting its PCM, with the same block
 * decoder (one thread; stores go straight to global memory).  Stops once a
 * block-end state equals the stored trajectory's (nothing after it can
 * change).  Returns true if it met the stored trajectory; otherwise stores
 * the new end state in e[q] and returns it in `exit`.
 */
template <int BITS, int CH>
__device__ bool
fix_chunk(const xa_dec_args &a, uint32_t q, uint2 s, uint2 &exit)
{
	typedef geo<BITS, CH> g;
	constexpr int G = g::G, OB = g::OB, WD = g::WD;
	int32_t p0[CH], p1[CH];
	xa_unpack_state(s.x, p0[0], p1[0]);
	if (CH == 2)
		xa_unpack_state(s.y, p0[CH - 1], p1[CH - 1]);
	const int64_t eblocks = a.eblocks;
	const int64_t b0 = (int64_t)q * a.C;
	int64_t b1 = b0 + a.C;
	if (b1 > eblocks)
		b1 = eblocks;
	auto none = [](int) {};

	/*
	 * Latency is what matters here (one busy lane per wave), so no load
	 * sits under a divergent branch -- hipcc drains vmcnt(0) right after
	 * such loads.  Every load is issued unconditionally with clamped
	 * indices (results past the chunk are never used), one group ahead:
	 * the next eblock's window and the next group's old block-end states.
	 * The decode lands in registers; only the stores are predicated.
	 */
	const int64_t ndw = (eblocks * g::EBSZ + 3) / 4;	/* source dwords */
	uint32_t buf[2][WD];
	/* old trajectory's block-end states (frames 30, 31) of a group, read
	 * before any rewrite; only used where b + 1 < eblocks */
	uint32_t old[G][CH], nxt[G][CH];
	auto rd = [&](uint32_t (*o_)[CH], int64_t bg) {
		auto one = [&](auto uc) {
			constexpr int u = decltype(uc)::value;
			const int64_t b = min(bg + u, eblocks - 1);
			const uint8_t *o = a.dst + b * OB;
			if (CH == 2) {
				uint2 f = *(const uint2 *)(o + 30 * 4);
				o_[u][0] = (f.y & 0xffffu) | (f.x << 16);
				o_[u][CH - 1] = (f.y >> 16) | (f.x & 0xffff0000u);
			} else {
				uint32_t f = *(const uint32_t *)(o + 30 * 2);
				o_[u][0] = (f >> 16) | (f << 16);
			}
		};
		sfor<0, G>::run(one);
	};
	bool met = false;
	load_window<BITS, CH, 0>(buf[0], a.src, b0);
	rd(old, b0);
	for (int64_t bg = b0; bg < b1; bg += G) {
		rd(nxt, bg + G);
		auto body = [&](auto uc) {
			constexpr int u = decltype(uc)::value;
			const int64_t b = bg + u;
			/* prefetch eblock b + 1's window (clamped: past the
			 * stream's end it is never used) */
			load_window_clamped<BITS, CH, (u + 1) % G>(buf[(u + 1) & 1],
			    a.src, b + 1, ndw);
			const bool act = !met && b < b1;
			int32_t q0[CH], q1[CH];
#pragma unroll
			for (int c = 0; c < CH; c++) {
				q0[c] = p0[c];
				q1[c] = p1[c];
			}
			uint32_t out[OB / 4] __attribute__((aligned(16)));
			(void)decode_eblock<BITS, CH, true, false, 64>(buf[u & 1],
			    g::woff(u), p0, p1, (uint8_t *)out, none);
			if (act) {
				uint8_t *d = a.dst + b * OB;
				if ((uint64_t)(b + 1) * OB <= a.pcm_bytes) {
#pragma unroll
					for (int i = 0; i < OB / 16; i++)
						((u32x4a *)d)[i] = ((const u32x4a *)out)[i];
				} else {
					/* the stream's cut last eblock */
#pragma unroll
					for (int k = 0; k < OB / 4; k++) {
						const uint64_t off = (uint64_t)b * OB + 4u * k;
						if (off + 4u <= a.pcm_bytes)
							*(uint32_t *)(a.dst + off) = out[k];
						else if (off < a.pcm_bytes)
							*(uint16_t *)(a.dst + off) =
							    (uint16_t)out[k];
					}
				}
			}
#pragma unroll
			for (int c = 0; c < CH; c++) {
				p0[c] = act ? p0[c] : q0[c];
				p1[c] = act ? p1[c] : q1[c];
			}
			if (act && b + 1 < eblocks) {
				bool m = true;
#pragma unroll
				for (int c = 0; c < CH; c++)
					m = m && xa_pack_state(p0[c], p1[c]) == old[u][c];
				met = m;
			}
		};
		sfor<0, G>::run(body);
		if (met)
			break;
#pragma unroll
		for (int u = 0; u < G; u++)
#pragma unroll
			for (int c = 0; c < CH; c++)
				old[u][c] = nxt[u][c];
	}
	if (met)
		return true;
	exit.x = xa_pack_state(p0[0], p1[0]);
	exit.y = CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u;
	a.e[q] = exit;
	return false;
}

/* binary min-heap over queue[0..n) (single thread) */
__device__ static void
heap_push(uint32_t *h, uint32_t &n, uint32_t v)
{
	uint32_t i = n++;
	while (i > 0) {
		uint32_t p = (i - 1) / 2;
		if (h[p] <= v)
			break;
		h[i] = h[p];
		i = p;
	}
	h[i] = v;
}

__device__ static uint32_t
heap_pop(uint32_t *h, uint32_t &n)
{
	const uint32_t top = h[0], v = h[--n];
	uint32_t i = 0;
	for (;;) {
		uint32_t c = 2 * i + 1;
		if (c >= n)
			break;
		if (c + 1 < n && h[c + 1] < h[c])
			c++;
		if (v <= h[c])
			break;
		h[i] = h[c];
		i = c;
	}
	if (n > 0)
		h[i] = v;
	return top;
}

/*
 * The sequential tail (one thread): drain the re-check queue in chunk order
 * (a heap, so even a pathological cascade costs O(n log n) bookkeeping),
 * then publish the status words and reset the control words.
 */
template <int BITS, int CH>
__device__ void
drain_tail(const xa_dec_args &a)
{
	const uint32_t nq = a.ctl[XA_CTL_NQ];
	uint32_t n = 0, tail = 0;
	for (uint32_t i = 0; i < nq; i++)
		heap_push(a.queue, n, a.queue[i]);
	while (n > 0) {
		const uint32_t q = heap_pop(a.queue, n);
		const uint2 s = a.e[q - 1], gq = a.g[q];
		if (s.x == gq.x && s.y == gq.y)
			continue;
		tail++;
		uint2 ex;
		const bool met = fix_chunk<BITS, CH>(a, q, s, ex);
		a.g[q] = s;
		if (!met && q + 1 < a.nchunks)
			heap_push(a.queue, n, q + 1);
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
	a.ctl[XA_CTL_TICKET] = 0;
}

/*
 * K2.  Verify every chunk boundary and repair mismatching chunks in
 * parallel; the last workgroup to finish then runs the sequential tail, so
 * the whole repair is one launch.  Per pass a workgroup checks
 * 256 * XA_FIX_CPT consecutive boundaries (a thread reads XA_FIX_CPT
 * consecutive e/g pairs), lists the mismatches in LDS, and then gives each
 * listed chunk a thread of its own: repairs of one wave run side by side,
 * so the pass costs the longest repair, not their sum.  Few, fat workgroups
 * keep the arrival ticket (one contended word) and the release fences
 * (only in workgroups that wrote) cheap.
 */
#ifndef XA_FIX_CPT
#define XA_FIX_CPT 4
#endif

template <int BITS, int CH>
__global__ __launch_bounds__(256) void
xa_decode_fix(xa_dec_args a)
{
	constexpr uint32_t SPAN = 256u * XA_FIX_CPT;
	__shared__ uint32_t last, nfix;
	__shared__ uint32_t fixq[SPAN];
	__shared__ uint2 fixs[SPAN];
	const uint32_t n = a.nchunks;
	const uint64_t *e64 = (const uint64_t *)a.e;
	const uint64_t *g64 = (const uint64_t *)a.g;
	bool wrote = false;
	for (uint32_t base = blockIdx.x * SPAN; base < n;
	    base += gridDim.x * SPAN) {
		if (threadIdx.x == 0)
			nfix = 0;
		__syncthreads();
		/* e[q-1] may be rewritten concurrently by chunk q-1's fixer;
		 * whichever value is read is recorded in g[q], and that fixer
		 * queues q for the tail, which re-checks it */
		const uint32_t t0 = base + threadIdx.x * XA_FIX_CPT;
		uint64_t ev[XA_FIX_CPT], gv[XA_FIX_CPT];
#pragma unroll
		for (int i = 0; i < XA_FIX_CPT; i++) {
			const uint32_t q = min(t0 + i, n - 1);
			ev[i] = __hip_atomic_load(&e64[q > 0 ? q - 1 : 0],
			    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			gv[i] = g64[q];
		}
#pragma unroll
		for (int i = 0; i < XA_FIX_CPT; i++) {
			const uint32_t q = t0 + i;
			if (q > 0 && q < n && ev[i] != gv[i]) {
				const uint32_t k = atomicAdd(&nfix, 1u);
				fixq[k] = q;
				fixs[k] = make_uint2((uint32_t)ev[i],
				    (uint32_t)(ev[i] >> 32));
			}
		}
		__syncthreads();
		const uint32_t nf = nfix;
		for (uint32_t k = threadIdx.x; k < nf; k += 256u) {
			const uint32_t q = fixq[k];
			const uint2 s = fixs[k];
			uint2 ex;
			const bool met = fix_chunk<BITS, CH>(a, q, s, ex);
			a.g[q] = s;
			wrote = true;
			if (!met && q + 1 < n) {
				uint32_t i = atomicAdd(&a.ctl[XA_CTL_NQ], 1u);
				a.queue[i] = q + 1;
			}
		}
		if (threadIdx.x == 0 && nf)
			atomicAdd(&a.ctl[XA_CTL_FIXED], nf);
		__syncthreads();
	}
	/* arrival ticket.  Release (MI355X_MICROARCH.md inter-workgroup
	 * recipe): every wave's stores done at the barrier, then lane 0's
	 * agent fence and its wait, then the ticket -- skipped by workgroups
	 * that stored nothing */
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	const int any = __syncthreads_or(wrote);
	if (threadIdx.x == 0) {
		if (any) {
			__threadfence();
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		}
		last = atomicAdd(&a.ctl[XA_CTL_TICKET], 1u) == gridDim.x - 1;
	}
	__syncthreads();
	if (!last || threadIdx.x != 0)
		return;
	/* acquire: this CU now sees every other workgroup's writes */
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	drain_tail<BITS, CH>(a);
}

/* ------------------------------------------------------------------ */

template <int BITS, int CH>
static hipError_t
launch(const xa_dec_args &a, unsigned variant, hipStream_t st, hipEvent_t ev0,
    hipEvent_t ev1)
{
	const unsigned per = 64u * XA_SPEC_WPB;
	const unsigned grid = (a.nchunks + per - 1) / per;
	unsigned grid2 = (a.nchunks + 256u * XA_FIX_CPT - 1) / (256u * XA_FIX_CPT);
	if (grid2 > 256u)
		grid2 = 256u;
	if (ev0 != NULL)
		(void)hipEventRecord(ev0, st);
	/* variant bit 0: SPLIT regions; bit 1: non-temporal output stores */
	switch (variant & 3u) {
	case 0:
		hipLaunchKernelGGL((xa_decode_spec<BITS, CH, false, 64 * CH, false>),
		    dim3(grid), dim3(per), 0, st, a);
		break;
	case 1:
		hipLaunchKernelGGL((xa_decode_spec<BITS, CH, true, 64 * CH, false>),
		    dim3(grid), dim3(per), 0, st, a);
		break;
	case 2:
		hipLaunchKernelGGL((xa_decode_spec<BITS, CH, false, 64 * CH, true>),
		    dim3(grid), dim3(per), 0, st, a);
		break;
	default:
		hipLaunchKernelGGL((xa_decode_spec<BITS, CH, true, 64 * CH, true>),
		    dim3(grid), dim3(per), 0, st, a);
		break;
	}
	if (ev1 != NULL)
		(void)hipEventRecord(ev1, st);
	hipLaunchKernelGGL((xa_decode_fix<BITS, CH>), dim3(grid2), dim3(256), 0,
	    st, a);
	return hipGetLastError();
}

hipError_t
xa_decode_launch(const xa_dec_args &a, unsigned bits, unsigned ch,
    unsigned variant, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1)
{
	if (ch == 1) {
		if (bits == 8)
			return launch<8, 1>(a, variant, st, ev0, ev1);
		if (bits == 6)
			return launch<6, 1>(a, variant, st, ev0, ev1);
		return launch<4, 1>(a, variant, st, ev0, ev1);
	}
	if (bits == 8)
		return launch<8, 2>(a, variant, st, ev0, ev1);
	if (bits == 6)
		return launch<6, 2>(a, variant, st, ev0, ev1);
	return launch<4, 2>(a, variant, st, ev0, ev1);
}
