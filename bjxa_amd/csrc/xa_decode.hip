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
 * owns two LDS buffers and alternates them group by group:
 *  - input: the group of each of its 64 chunks, fetched by LDS-DMA with the
 *    64 segments concatenated, so every DMA instruction fills 1 KiB of LDS
 *    from a few 144-B runs of the stream (instead of 64 scattered 16-B
 *    pieces, which saturated the texture addresser).  A lane copies its
 *    segment to VGPRs and the next group's DMA is issued into the other
 *    buffer at once, so it lands while this group decodes.
 *  - output: the group's PCM is staged 128 B per lane in the buffer just
 *    consumed and stored so that each instruction covers 8 whole lines.
 *    The wait for the next group's DMA is vmcnt(16): it leaves this
 *    group's 16 stores in flight.
 * Predictor: stereo runs both channels as the two halves of packed-f32
 * instructions (xa_step_lr), mono a single f32 chain (xa_step_f); both are
 * exact (xa_common.h).
 */
#include "xa_kern.h"

#ifndef XA_SPEC_WPB
#define XA_SPEC_WPB 4		/* waves per workgroup */
#endif
#ifndef XA_FIX_PF
#define XA_FIX_PF 4		/* repair windows in flight per lane */
#endif


/*
 * Store the wave's staged LB-byte lines: line j belongs to chunk
 * wchunk0 + j (whose PCM starts at wstart_b + j * chunk_bytes) and goes to
 * byte `rel_off` of that chunk's PCM.  Lane l
 * stores piece l % P of lines l / P + (64 / P) i (P = LB / 16 pieces per
 * line).  Wave-uniform fast path when every line is whole; a predicated
 * copy of it when the stream ends inside the wave on a 16-B boundary;
 * otherwise (a cut last block) per-piece bounds and a 2-byte tail.
 */
template <int LB, bool NT>
__device__ __forceinline__ void
store_lines(const xa_dec_args &a, const uint8_t *obuf, int lane,
    uint32_t wchunk0, uint64_t wstart_b, uint32_t chunk_bytes, uint32_t rel_off,
    bool wave_full, bool clean, uint8_t *gbase, const uint8_t *lbase)
{
	constexpr int LINE = LB + 16, P = LB / 16, LPI = 64 / P;
#ifdef XA_DBG_NOSTORE
	/* diagnostic build only (no output) */
	if (wave_full)
		return;
#endif
	if (wave_full) {
#ifdef XA_DBG_CONTIG
		/* diagnostic build only (wrong layout): the same bytes, each
		 * store instruction writing 1 KiB contiguously inside the
		 * wave's own region */
		{
			uint8_t *wp = a.dst + wstart_b + (uint64_t)rel_off * 64u +
			    (uint64_t)lane * 16u;
#pragma unroll
			for (int i = 0; i < P; i++) {
				const u32x4a v = *(const u32x4a *)(lbase +
				    i * LPI * LINE);
				__builtin_nontemporal_store(v,
				    (u32x4a *)(wp + i * 1024));
			}
			return;
		}
#endif
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
	if (clean) {
		/* the stream ends in this wave but its PCM is a whole number of
		 * 16-B pieces: the fast path with each piece predicated on lying
		 * in the stream (pieces of chunks past the end lie beyond it) */
		uint8_t *gp = gbase + rel_off;
		const uint8_t *end = a.dst + a.pcm_bytes;
		const uint64_t istride = (uint64_t)LPI * chunk_bytes;
#pragma unroll
		for (int i = 0; i < P; i++) {
			const u32x4a v = *(const u32x4a *)(lbase + i * LPI * LINE);
			uint8_t *q = gp + i * istride;
			if (q + 16 <= end) {
				if (NT)
					__builtin_nontemporal_store(v, (u32x4a *)q);
				else
					*(u32x4a *)q = v;
			}
		}
		return;
	}
	/* launder the inputs so none of this rare path's address arithmetic
	 * is hoisted out of the caller's loops (it would pin ~100 VGPRs) */
	uint32_t wc = wchunk0, nch = a.nchunks, cb = chunk_bytes, ro = rel_off;
	uint64_t lim = a.pcm_bytes, wsb = wstart_b;
	uint8_t *dst = a.dst;
	asm volatile("" : "+v"(wc), "+v"(nch), "+v"(cb), "+v"(ro), "+v"(lim),
	    "+v"(dst), "+v"(wsb));
#pragma nounroll
	for (int i = 0; i < P; i++) {
		const int j = i * LPI + lane / P, pc = lane % P;
		const uint32_t cj = wc + (uint32_t)j;
		const uint64_t off = wsb + (uint64_t)j * cb + ro + (uint64_t)pc * 16u;
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
 * K1.  One lane per chunk, XA_SPEC_WPB waves per workgroup.
 *  LB  output bytes per lane per store phase (64, 128 or 256; a phase may
 *      span eblocks)
 *  NT  non-temporal PCM stores
 * One LDS region per wave serves both directions: a group's input is
 * copied to VGPRs, then its output lines are staged and stored, then the
 * next group's DMA is issued.  (Separate regions with the DMA issued before
 * the decode and a counted vmcnt measured no faster)
 */

/*
 * K1 body: one wave decodes chunks wchunk0 .. wchunk0+63 of stream `a`
 * (wave-uniform) with two-group input runs.  A lane's input for a
 * "super-step" (two groups, 2G eblocks) is one contiguous run of 8*GDW
 * bytes.  The runs of half a wave (32 lanes) land together in one LDS
 * buffer, so a DMA instruction reads two runs of ~264 B instead of seven
 * 144-B segments (fewer, longer DRAM bursts: the K1 skeleton of
 * tools/pattern_probe.hip runs 4.5 % faster this way), and each lane keeps
 * its run in VGPRs.  The next super-step's two halves land while this one
 * decodes: half 0 before the first group, half 1 before the second, each
 * wait leaving the previous group's 16 stores in flight.  Output lines are
 * staged in a separate region as before.
 */
#define XA_NST 16	/* store instructions per group (G * OB / 16) */

template <int BITS, int CH> struct geo2 {
	typedef geo<BITS, CH> g;
	static constexpr int RD = 2 * g::GDW;			/* dwords per run */
	static constexpr int SLOT = (RD * 4 + 15) / 16 * 16;	/* LDS bytes per run */
	static constexpr int NPR = SLOT / 16;			/* 16-B pieces per run */
	static constexpr int NI = (32 * NPR + 63) / 64;		/* DMA instructions per half */
	static constexpr int LAST = 32 * NPR - 64 * (NI - 1);	/* lanes of the last one */
	static constexpr int HALF = 32 * SLOT;
};

template <int BITS, int CH, int LB> struct spec_lds2 {
	static constexpr int LINE = LB + 16;
	static constexpr int REGION = geo2<BITS, CH>::HALF + 64 * LINE;
};

/*
 * Stage the runs of half h of the wave (chunks 32h .. 32h+31 of the wave)
 * that start `rel` eblocks into their chunks.  Piece k of the landing image
 * is run k / NPR, bytes 16 (k % NPR) ... (voff).  Runs that reach outside
 * the stream (the grid's first and last waves) take dword pieces, each
 * clamped into the stream whole (the dword holding the stream's last byte
 * is read whole, nothing past it); their lanes never decode those bytes.
 * LDS-DMA facts (tools/dma_probe.hip): 16-B pieces land packed lane-linear
 * in LDS even from 4-B aligned sources; 12-B pieces land at a 16-B lane
 * stride, so runs are read rounded up to 16 B (SLOT).
 */
template <int BITS, int CH>
__device__ __forceinline__ void
stage_half(const xa_dec_args &a, uint8_t *land, int lane, int64_t wstart,
    uint32_t Cw, int h, int64_t rel, const uint32_t *voff)
{
	typedef geo<BITS, CH> g;
	typedef geo2<BITS, CH> g2;
	const int64_t c0 = wstart + (int64_t)h * 32 * Cw;
	const int64_t e_first = c0 + rel;
	const int64_t e_end = c0 + 31 * (int64_t)Cw + rel + 2 * g::G;
	if (e_first >= 0 && e_end * g::EBSZ + (g2::SLOT - 4 * g2::RD) <=
	    (int64_t)a.eblocks * g::EBSZ) {
		const uint8_t *base = a.src + (size_t)e_first * g::EBSZ;
#pragma unroll
		for (int i = 0; i < g2::NI; i++)
			if (i < g2::NI - 1 || lane < g2::LAST)
				dma<16>(base + voff[i], land + i * 1024);
		return;
	}
	uint32_t C = Cw, neb = a.eblocks;
	int64_t r = c0 + rel;
	const uint8_t *src = a.src;
	asm volatile("" : "+v"(C), "+v"(neb), "+v"(r), "+v"(src));
	constexpr int SD = g2::SLOT / 4;
	const int64_t last = ((int64_t)neb * g::EBSZ - 1) & ~(int64_t)3;
#pragma nounroll
	for (int i = 0; i < (32 * SD + 63) / 64; i++) {
		const int k = i * 64 + lane, run = k / SD, off = k % SD;
		if (k >= 32 * SD)
			continue;
		int64_t byte = ((int64_t)run * C + r) * g::EBSZ + off * 4;
		byte = byte < 0 ? 0 : (byte > last ? last : byte);
		dma<4>(src + byte, land + i * 256);
	}
}

template <int BITS, int CH, int LB, bool NT>
__device__ __forceinline__ void
spec_wave2(const xa_dec_args &a, uint8_t *region, const uint32_t wchunk0,
    const uint32_t pace_every)
{
	typedef geo<BITS, CH> g;
	typedef geo2<BITS, CH> g2;
	constexpr int G = g::G, OB = g::OB, EBSZ = g::EBSZ, GDW = g::GDW;
	constexpr int RD = g2::RD, LINE = LB + 16;
	static_assert(G * OB / 16 == XA_NST, "store count per group");

	const int lane = threadIdx.x & 63;
	uint8_t *land = region, *ost = region + g2::HALF;
	const uint32_t chunk = wchunk0 + lane;
	const int64_t eblocks = a.eblocks;
	const bool lng = wchunk0 < a.nlong;
	const uint32_t Cw = a.C + (lng ? a.dlong : 0u);
	const int64_t wstart = chunk_start(a, wchunk0);
	const int64_t b0 = wstart + (int64_t)lane * Cw;
	const int W = (int)(lng ? a.Wlong : a.W);
	/* super-steps: NW of warm-up, then NC of the chunk (W and Cw are
	 * multiples of 2G, the host plans them so) */
	const int NW = W / (2 * G), NS = NW + (int)Cw / (2 * G);

	uint32_t voff[g2::NI];
#pragma unroll
	for (int i = 0; i < g2::NI; i++) {
		const int k = i * 64 + lane;
		voff[i] = (uint32_t)(k / g2::NPR) * Cw * EBSZ +
		    (uint32_t)(k % g2::NPR) * 16u;
	}

	int32_t p0[CH], p1[CH];
#pragma unroll
	for (int c = 0; c < CH; c++) {
		if (b0 - W <= 0)	/* the stream start: the caller's state */
			xa_unpack_state(a.init[c], p0[c], p1[c]);
		else
			p0[c] = p1[c] = 0;
	}
	uint32_t gst[2] = { 0u, 0u };

	const uint32_t chunk_bytes = Cw * OB;
	const uint64_t wstart_b = (uint64_t)wstart * OB;
	constexpr int P = LB / 16;
	uint8_t *gbase = a.dst + wstart_b + (uint64_t)(lane / P) * chunk_bytes +
	    (lane % P) * 16;
	const uint8_t *lbase = ost + (lane / P) * LINE + (lane % P) * 16;
	uint8_t *line = ost + lane * LINE;
	const uint64_t full_blocks = a.pcm_bytes / OB;
	const bool wave_full = wchunk0 + 63u < a.nchunks &&
	    (uint64_t)(wstart + 64 * (int64_t)Cw) <= full_blocks;
	const bool clean = (a.pcm_bytes & 15u) == 0;
	auto none = [](int) {};

	/* copy this lane's run out of the landing buffer (half h only) */
	auto take = [&](int h, uint32_t *dst) {
		if ((lane >> 5) == h) {
			const uint32_t *m = (const uint32_t *)(land +
			    (lane & 31) * g2::SLOT);
#pragma unroll
			for (int i = 0; i < RD; i++)
				dst[i] = m[i];
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	};
	auto rel_of = [&](int S) -> int64_t { return (int64_t)S * 2 * G - W; };
	/* wait for the DMA issued just before decoding group gi: only that
	 * group's stores are younger, when it stored on the fast path */
	auto wait_after = [&](int gi) {
#ifndef XA_DBG_NOSTORE
		if (gi >= 2 * NW && wave_full)
			asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA_NST) : "memory");
		else
#endif
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	};

	/* decode group hh (0/1) of super-step S from run r */
	auto group = [&](const uint32_t *r, int S, auto hc) {
		constexpr int hh = decltype(hc)::value;
		if (S < NW) {
			auto body = [&](auto uc) {
				constexpr int u = decltype(uc)::value;
				const int64_t b = b0 + rel_of(S) + hh * G + u;
				if (b >= 0 && b < eblocks)
					(void)decode_eblock<BITS, CH, false, true, 64>(r,
					    hh * 4 * GDW + u * EBSZ, p0, p1, line, none);
			};
			sfor<0, G>::run(body);
			return;
		}
		const int s0 = (S - NW) * 2 * G + hh * G;
		auto body = [&](auto uc) {
			constexpr int u = decltype(uc)::value;
			const int64_t b = b0 + s0 + u;
			auto flush = [&](int h) {
				wave_lds_sync();
				__builtin_amdgcn_s_setprio(1);
				store_lines<LB, NT>(a, ost, lane, wchunk0, wstart_b,
				    chunk_bytes, (uint32_t)s0 * OB + (uint32_t)LB * h,
				    wave_full, clean, gbase, lbase);
				__builtin_amdgcn_s_setprio(0);
				wave_lds_sync();
			};
			const bool act = b < eblocks;
			int32_t q0[CH], q1[CH];
#pragma unroll
			for (int c = 0; c < CH; c++) {
				q0[c] = p0[c];
				q1[c] = p1[c];
			}
			uint32_t bad = decode_eblock<BITS, CH, true, true, LB,
			    u * 4 * CH>(r, hh * 4 * GDW + u * EBSZ, p0, p1, line,
			    flush);
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
	};

	/* wave priority: a wave that has its next run landed takes the issue
	 * slot for its LDS reads and DMA ahead of the other wave's decode VALU
	 * (2), and for its PCM stores (1), so the memory pipeline sees the
	 * next requests sooner (C3 spec -1.3 %, C2 -1.6 %; the stores above
	 * or level with the DMA measured no better than without priorities) */
	auto prio = [](auto pc) {
#ifndef XA_NOPRIO
		__builtin_amdgcn_s_setprio(decltype(pc)::value);
#endif
	};
	/* one super-step from run `cur`, landing the next one into `nxt` */
	/*
	 * Pacing: every `pace_every` groups the workgroup's waves wait for
	 * each other (a bare s_barrier, no memory fence: the LDS regions are
	 * per wave).  Left to themselves the waves drift apart -- issue
	 * arbitration favours the older ones -- and the early finishers leave
	 * their CU with fewer requests in flight for the rest of the kernel;
	 * paced, they all stream to the end (C3 spec -4 %, C2 -4.5 %,
	 * DESIGN.md §5).  The host sets pace_every (0 = off) only when every
	 * wave of the workgroup runs the same number of groups.
	 */
	auto pace = [&](int gi) {
		if (pace_every != 0u && (uint32_t)gi % pace_every == 0u)
			__builtin_amdgcn_s_barrier();
	};
	auto step = [&](int S, uint32_t *cur, uint32_t *nxt) {
		pace(2 * S);
		if (S == NW) {
			gst[0] = xa_pack_state(p0[0], p1[0]);
			gst[1] = CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u;
		}
		const bool more = S + 1 < NS;
		if (more) {
			if (S == 0)
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			else
				wait_after(2 * S - 1);
			prio(std::integral_constant<int, 2>());
			take(0, nxt);
			stage_half<BITS, CH>(a, land, lane, wstart, Cw, 1,
			    rel_of(S + 1), voff);
			prio(std::integral_constant<int, 0>());
		}
		asm volatile("" ::: "memory");
		group(cur, S, std::integral_constant<int, 0>());
		/* the staged lines have been read back */
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		if (more) {
			wait_after(2 * S);
			prio(std::integral_constant<int, 2>());
			take(1, nxt);
			if (S + 2 < NS)
				stage_half<BITS, CH>(a, land, lane, wstart, Cw, 0,
				    rel_of(S + 2), voff);
			prio(std::integral_constant<int, 0>());
		}
		asm volatile("" ::: "memory");
		pace(2 * S + 1);
		group(cur, S, std::integral_constant<int, 1>());
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	};

#ifdef XA_DBG_TIMES
	/* diagnostic build only: per-wave timeline (s_memrealtime, 100 MHz) --
	 * start, end of warm-up, end -- and the XCD/SE/CU of the wave, written
	 * into the second half of the re-check queue (tools/wave_times.py) */
	uint32_t *trec = a.queue + a.nchunks + (wchunk0 / 64u) * 4u;
	const uint32_t t_start = (uint32_t)__builtin_amdgcn_s_memrealtime();
	uint32_t t_warm = t_start;
#endif
	uint32_t A[RD], B[RD];
	/* prologue: super-step 0 into A, half 0 of super-step 1 in flight */
	stage_half<BITS, CH>(a, land, lane, wstart, Cw, 0, rel_of(0), voff);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(0, A);
	stage_half<BITS, CH>(a, land, lane, wstart, Cw, 1, rel_of(0), voff);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(1, A);
	if (NS > 1)
		stage_half<BITS, CH>(a, land, lane, wstart, Cw, 0, rel_of(1),
		    voff);
	for (int S = 0; S < NS; S += 2) {
#ifdef XA_DBG_TIMES
		if (S == NW)
			t_warm = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
		step(S, A, B);
		if (S + 1 < NS)
			step(S + 1, B, A);
	}
#ifdef XA_DBG_TIMES
	{
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		const uint32_t t_end = (uint32_t)__builtin_amdgcn_s_memrealtime();
		/* HW_ID (id 4): cu 11:8, se 15:13; XCC_ID (id 20) */
		const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
		const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
		if (lane == 0) {
			trec[0] = t_start;
			trec[1] = t_warm;
			trec[2] = t_end;
			trec[3] = (xcc & 15u) << 16 | ((hw >> 13) & 7u) << 8 |
			    ((hw >> 8) & 15u) << 4 | ((hw >> 4) & 3u);
		}
	}
#endif
	if (NS == NW) {	/* empty chunk (never planned) */
		gst[0] = xa_pack_state(p0[0], p1[0]);
		gst[1] = CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u;
	}
	if (chunk < a.nchunks) {
		a.g[chunk] = make_uint2(gst[0], gst[1]);
		a.e[chunk] = make_uint2(xa_pack_state(p0[0], p1[0]),
		    CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u);
	}
}

/* K1 for one stream: wave w of the grid takes chunks 64w .. 64w+63 */
template <int BITS, int CH, int LB, bool NT>
__global__ __launch_bounds__(64 * XA_SPEC_WPB, 8 / XA_SPEC_WPB) void
xa_decode_spec(xa_dec_args a)
{
	/* the wave index is wave-uniform; say so, so that LDS bases and the
	 * DMA source base live in SGPRs */
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	typedef spec_lds2<BITS, CH, LB> L;
	__shared__ __attribute__((aligned(16))) uint8_t
	    lds[XA_SPEC_WPB * L::REGION];
	/* every wave of the workgroup has the same chunk length unless the
	 * balanced plan's long/short edge falls inside it */
	const uint32_t first = blockIdx.x * (64u * XA_SPEC_WPB);
	const bool uniform = first >= a.nlong ||
	    first + 64u * (XA_SPEC_WPB - 1) < a.nlong;
	spec_wave2<BITS, CH, LB, NT>(a, lds + wv * L::REGION, first + wv * 64u,
	    uniform ? a.pace : 0u);
}

/* ------------------------------------------------------------------ */
/* repair path                                                          */

/*
 * Re-decode chunk q from the state s (s.x: channel 0, s.y: channel 1),
 * rewriting its PCM, on one lane: the eblock goes through K1's own
 * decode_eblock (stereo: both channels in one packed-f32 instruction stream,
 * 11 VALU per frame, with the output frame packed by the step itself; mono:
 * the f32 chain), so repaired PCM is K1's arithmetic bit for bit.  Stops
 * once a block-end state equals the stored trajectory (frames 30/31 of the
 * old PCM) in every channel: nothing after it can change.  Returns true if
 * it met the trajectory; otherwise stores the chunk's new exit state in
 * e[q] and returns it in `exit`.
 *
 * The repair is one serial chain per chunk, so its time is its instruction
 * count: the earlier lane-per-channel integer form issued ~467 VALU per
 * repaired block (a lane pair per stereo chunk, plus the frame shuffle
 * between them); this one ~11 per frame.
 *
 * No load sits under a branch (hipcc drains vmcnt(0) right after such
 * loads): the windows and old end states of the blocks XA_FIX_PF ahead are
 * fetched every iteration with clamped addresses.  BUF (one stream per
 * launch, under 4 GiB of XA): the window comes through a buffer descriptor
 * of the stream, whose range check returns 0 past the end, instead of
 * per-dword 64-bit clamps.
 */
template <int BITS, int CH, bool BUF = false>
__device__ __forceinline__ bool
fix_chunk(const xa_dec_args &a, uint32_t q, uint2 s, uint2 &exit)
{
	typedef geo<BITS, CH> g;
	constexpr int EBSZ = g::EBSZ, OB = g::OB;
	constexpr int WN = (EBSZ + 3) / 4;	/* dwords of one eblock */
	int32_t p0[CH], p1[CH];
	xa_unpack_state(s.x, p0[0], p1[0]);
	if (CH == 2)
		xa_unpack_state(s.y, p0[CH - 1], p1[CH - 1]);
	const int64_t eblocks = a.eblocks;
	const int64_t b0 = chunk_start(a, q);
	int64_t b1 = chunk_start(a, q + 1);
	if (b1 > eblocks)
		b1 = eblocks;
	const int64_t ndw = (eblocks * EBSZ + 3) / 4;
	const uint32_t *src = (const uint32_t *)a.src;
	/* q >= 1, so the stream has whole blocks (nfull >= b0 >= 16) */
	const int64_t nfull = (int64_t)(a.pcm_bytes / OB);

	__amdgpu_buffer_rsrc_t rs;
	if constexpr (BUF) {
		const uint64_t sp = (uint64_t)a.src;
		const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)sp);
		const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(sp >> 32));
		const uint32_t nb = __builtin_amdgcn_readfirstlane((uint32_t)(ndw * 4));
		rs = __builtin_amdgcn_make_buffer_rsrc(
		    (void *)(((uint64_t)hi << 32) | lo), 0, (int)nb, 0x00020000);
	}
	/* the WN + 1 dwords holding eblock b */
	auto fetch = [&](uint32_t *r, int64_t b) {
		const int64_t d0 = (b * EBSZ) >> 2;
		if constexpr (BUF) {
			const uint32_t o = (uint32_t)d0 * 4u;
#pragma unroll
			for (int i = 0; i <= WN; i++)
				r[i] = __builtin_amdgcn_raw_buffer_load_b32(rs,
				    (int)(o + 4u * i), 0, 0);
		} else {
#pragma unroll
			for (int i = 0; i <= WN; i++)
				r[i] = src[min(d0 + i, ndw - 1)];
		}
	};
	/* old end state of block b: its PCM frames 30 and 31 as stored (raw, so
	 * nothing uses the loaded words before the block's compare, PF blocks
	 * later), clamped to the last whole block: a stream whose last block is
	 * cut is never read past its PCM */
	auto old_state = [&](int64_t b) {
		const uint8_t *p = a.dst + min(b, nfull - 1) * OB;
		if (CH == 2)
			return *(const uint2 *)(p + 120);
		return make_uint2(*(const uint32_t *)(p + 60), 0u);
	};
	/* does the state in p0/p1 equal the raw frames f? */
	auto same_state = [&](uint2 f) {
		if (CH == 2)
			return f.x == (((uint32_t)p1[0] & 0xffffu) | ((uint32_t)p1[CH - 1] << 16)) &&
			    f.y == (((uint32_t)p0[0] & 0xffffu) | ((uint32_t)p0[CH - 1] << 16));
		return f.x == (((uint32_t)p1[0] & 0xffffu) | ((uint32_t)p0[0] << 16));
	};
	auto none = [](int) {};
	/* decode eblock b from its window r, PCM to `out` (16-B pieces) */
	auto decode = [&](const uint32_t *r, int64_t b, uint8_t *out) {
		const uint32_t o = (uint32_t)(b * EBSZ) & 3u;
		uint32_t w[WN];
#pragma unroll
		for (int i = 0; i < WN; i++)
			w[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], o);
		(void)decode_eblock<BITS, CH, true, false, OB>(w, 0, p0, p1, out,
		    none);
	};

	constexpr int PF = XA_FIX_PF;
	const int64_t bf = min(b1, nfull);
	uint32_t ring[PF][WN + 1];
	uint2 rold[PF];
#pragma unroll
	for (int j = 0; j < PF; j++) {
		fetch(ring[j], b0 + j);
		rold[j] = old_state(b0 + j);
	}
	/* every slot's loaded words are first used PF blocks after their load,
	 * in straight-line code under the lane's `act` mask, so the waits are
	 * counted ones (no join block consumes a pending load) */
	bool met = false, act = b0 < bf;
	int64_t b = b0;
	while (act) {
#pragma unroll
		for (int j = 0; j < PF; j++) {
			if (act) {
				decode(ring[j], b, a.dst + (uint64_t)b * OB);
				const bool m = b + 1 < eblocks && same_state(rold[j]);
				fetch(ring[j], b + PF);
				rold[j] = old_state(b + PF);
				b++;
				met = m;
				act = !m && b < bf;
			}
		}
	}
	if (!met && b < b1) {
		/* b == eblocks - 1, PCM cut short: no later block to meet */
		uint32_t raw[WN + 1];
		uint32_t F[OB / 4] __attribute__((aligned(16)));
		fetch(raw, b);
		decode(raw, b, (uint8_t *)F);
		const uint64_t off = (uint64_t)b * OB;
		uint8_t *d = a.dst + off;
#pragma unroll
		for (int k = 0; k < OB / 4; k++) {
			if (off + 4u * k + 4u <= a.pcm_bytes)
				((uint32_t *)d)[k] = F[k];
			else if (off + 4u * k < a.pcm_bytes)
				((uint16_t *)d)[2 * k] = (uint16_t)F[k];
		}
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
 * The sequential tail (lane 0 of one wave): drain the re-check queue in chunk
 * order (a heap, so even a pathological cascade costs O(n log n)
 * bookkeeping), then publish the status words and reset the control words.
 * Queue entries are >= 1, so 0 ends the loop.
 */
template <int BITS, int CH, bool BUF>
__device__ __forceinline__ void
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
#ifdef XA_DBG_NOTAIL
		/* timing diagnostic only: leaves cascaded chunks unrepaired */
		continue;
#endif
		uint2 ex;
		const bool met = fix_chunk<BITS, CH, BUF>(a, q, s, ex);
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
	a.status[XA_ST_CHUNKS] = a.rep_chunks ? a.rep_chunks : a.nchunks;
	a.status[XA_ST_C] = a.rep_C ? a.rep_C : a.C;
	a.status[XA_ST_W] = a.W;
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
#define XA_FIX_CPT 2
#endif
#ifndef XA_FIXB_MAXWG
#define XA_FIXB_MAXWG 256u	/* batch K2 workgroups at most */
#endif
#ifndef XA_FIXB_WPB
#define XA_FIXB_WPB 4u		/* batch K2 waves per workgroup */
#endif
#ifndef XA_FIX_REL
#define XA_FIX_REL 0
#endif

/* K2's release before the arrival ticket */
__device__ __forceinline__ void
xa_fix_release()
{
#if XA_FIX_REL == 1
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#else
	__threadfence();
#endif
}


template <int BITS, int CH, bool BUF>
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
		/* a lane per listed chunk */
		for (uint32_t k = threadIdx.x; k < nf; k += 256u) {
			const uint32_t q = fixq[k];
			const uint2 s = fixs[k];
			uint2 ex;
			const bool met = fix_chunk<BITS, CH, BUF>(a, q, s, ex);
			wrote = true;
			a.g[q] = s;
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
			xa_fix_release();
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
	drain_tail<BITS, CH, BUF>(a);
}

/* ------------------------------------------------------------------ */

/* K2 over a.nchunks chunks of a.C eblocks */
template <int BITS, int CH>
static hipError_t
fix_launch(const xa_dec_args &a, hipStream_t st)
{
	unsigned grid2 = (a.nchunks + 256u * XA_FIX_CPT - 1) / (256u * XA_FIX_CPT);
	if (grid2 > 256u)
		grid2 = 256u;
#ifdef XA_FIX_NOBUF
	const bool buf = false;
#else
	/* buffer-descriptor windows need 32-bit byte offsets */
	const bool buf = (uint64_t)a.eblocks * geo<BITS, CH>::EBSZ <
	    (1ull << 32) - 256u;
#endif
	if (buf)
		hipLaunchKernelGGL((xa_decode_fix<BITS, CH, true>), dim3(grid2),
		    dim3(256), 0, st, a);
	else
		hipLaunchKernelGGL((xa_decode_fix<BITS, CH, false>), dim3(grid2),
		    dim3(256), 0, st, a);
	return hipGetLastError();
}

hipError_t
xa_decode_fix_launch(const xa_dec_args &a, unsigned bits, unsigned ch,
    hipStream_t st)
{
	if (ch == 1) {
		if (bits == 8)
			return fix_launch<8, 1>(a, st);
		if (bits == 6)
			return fix_launch<6, 1>(a, st);
		return fix_launch<4, 1>(a, st);
	}
	if (bits == 8)
		return fix_launch<8, 2>(a, st);
	if (bits == 6)
		return fix_launch<6, 2>(a, st);
	return fix_launch<4, 2>(a, st);
}

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
	/* variant bit 1: non-temporal PCM stores; bits 2-3: bytes per lane
	 * per store phase (0: one eblock, 1: 128; 256-B phases, measured
	 * slower, no longer fit two double-buffered workgroups per CU) */
#define SPEC(LB, NT) hipLaunchKernelGGL((xa_decode_spec<BITS, CH, LB, NT>), \
    dim3(grid), dim3(per), 0, st, a)
	const bool nt = (variant & 2u) != 0;
	switch ((variant >> 2) & 3u) {
	case 1:
		if (nt) SPEC(128, true); else SPEC(128, false);
		break;
	default:
		if (nt) SPEC(64 * CH, true); else SPEC(64 * CH, false);
		break;
	}
#undef SPEC
	if (ev1 != NULL)
		(void)hipEventRecord(ev1, st);
#if !defined(XA_DBG_STEP) && !defined(XA_DBG_NOSTORE) && !defined(XA_DBG_CONTIG)
	const hipError_t e2 = fix_launch<BITS, CH>(a, st);
	if (e2 != hipSuccess)
		return e2;
#endif
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

/* ------------------------------------------------------------------ */
/* batched decode: many streams, mixed formats                          */

/* f(BITS, CH) as integral constants for fmt = bits | channels << 8 */
template <typename F>
__device__ __forceinline__ void
with_format(uint32_t fmt, F &&f)
{
	typedef std::integral_constant<int, 1> c1;
	typedef std::integral_constant<int, 2> c2;
	switch (fmt) {
	case 8 | 2 << 8:
		f(std::integral_constant<int, 8>(), c2());
		break;
	case 6 | 2 << 8:
		f(std::integral_constant<int, 6>(), c2());
		break;
	case 4 | 2 << 8:
		f(std::integral_constant<int, 4>(), c2());
		break;
	case 8 | 1 << 8:
		f(std::integral_constant<int, 8>(), c1());
		break;
	case 6 | 1 << 8:
		f(std::integral_constant<int, 6>(), c1());
		break;
	default:
		f(std::integral_constant<int, 4>(), c1());
		break;
	}
}

/* the single-stream argument block of stream `sid` of a batch */
__device__ __forceinline__ xa_dec_args
batch_stream_args(const xa_batch_args &b, uint32_t sid)
{
	const xa_batch_stream &d = b.streams[sid];
	xa_dec_args a;
	a.src = d.src;
	a.dst = d.dst;
	a.pcm_bytes = d.pcm_bytes;
	a.eblocks = d.eblocks;
	a.nchunks = d.nchunks;
	a.C = d.C;
	/* two chunk lengths: the short chunks' warm-up makes their lanes'
	 * super-step count that of the long ones */
	a.W = d.nlong ? d.Wlong + d.dlong : b.W;
	a.nlong = d.nlong;
	a.dlong = d.dlong;
	a.Wlong = d.nlong ? d.Wlong : b.W;
	a.pace = 0;	/* the batch kernel decides per workgroup */
	a.rep_C = a.rep_chunks = 0;
	a.init[0] = d.init[0];
	a.init[1] = d.init[1];
	a.g = b.g + d.cbase;
	a.e = b.e + d.cbase;
	a.queue = b.queue;
	a.ctl = b.sctl + sid * XA_SCTL_WORDS;	/* [XA_CTL_ERR] == [XA_SCTL_ERR] */
	a.status = b.status + sid * XA_ST_WORDS;
	return a;
}

template <int LB> struct batch_lds {
	static constexpr int m(int x, int y) { return x > y ? x : y; }
	/* one region per wave (landing buffer + output stage), the
	 * largest over the formats */
	static constexpr int REGION = m(m(m(spec_lds2<8, 2, LB>::REGION,
	    spec_lds2<8, 1, LB>::REGION), m(spec_lds2<6, 2, LB>::REGION,
	    spec_lds2<6, 1, LB>::REGION)), m(spec_lds2<4, 2, LB>::REGION,
	    spec_lds2<4, 1, LB>::REGION));
};

/* K1 over a batch: wave w decodes 64 chunks of stream wstream[w] with that
 * stream's format (wave-uniform dispatch, no divergence) */
template <int LB, bool NT>
__global__ __launch_bounds__(64 * XA_SPEC_WPB, 8 / XA_SPEC_WPB) void
xa_decode_spec_batch(xa_batch_args b)
{
	__shared__ __attribute__((aligned(16))) uint8_t
	    lds[XA_SPEC_WPB * batch_lds<LB>::REGION];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint32_t w = blockIdx.x * XA_SPEC_WPB + wv;
	/* lockstep (spec_wave2) only when all the workgroup's waves exist
	 * and run the same number of super-steps: same chunk length and
	 * channel count */
	const uint32_t w0 = blockIdx.x * XA_SPEC_WPB;
	bool lockstep = b.pace != 0u && w0 + XA_SPEC_WPB <= b.nwaves;
	if (lockstep) {
		/* a wave's lane length (warm-up + chunk: the same for both
		 * chunk lengths of a stream) and channel count */
		auto shape = [&](uint32_t wk) {
			const xa_batch_stream &d = b.streams[b.wstream[wk]];
			const uint32_t len = d.nlong == 0u ? b.W + d.C :
			    d.Wlong + d.dlong + d.C;
			return len | (d.fmt >> 8) << 24;
		};
		const uint32_t s0 = shape(w0);
		for (int k = 1; k < XA_SPEC_WPB; k++)
			lockstep = lockstep && shape(w0 + k) == s0;
	}
	lockstep = __builtin_amdgcn_readfirstlane(lockstep);
	if (w >= b.nwaves)
		return;
	const uint32_t sid = __builtin_amdgcn_readfirstlane(b.wstream[w]);
	const xa_dec_args a = batch_stream_args(b, sid);
	const uint32_t fmt = __builtin_amdgcn_readfirstlane(b.streams[sid].fmt);
	const uint32_t wchunk0 = 64u * w -
	    __builtin_amdgcn_readfirstlane(b.streams[sid].cbase);
	uint8_t *region = lds + wv * batch_lds<LB>::REGION;
	with_format(fmt, [&](auto bc, auto cc) {
		spec_wave2<decltype(bc)::value, decltype(cc)::value, LB, NT>(a,
		    region, wchunk0, lockstep ? b.pace : 0u);
	});
}

/* fix_chunk in a stream's format (a per-lane switch: no generic lambda, so
 * the argument block stays in registers) */
__device__ __forceinline__ bool
fix_any(const xa_dec_args &a, uint32_t fmt, uint32_t q, uint2 s, uint2 &ex)
{
	switch (fmt) {
	case 8 | 2 << 8:
		return fix_chunk<8, 2>(a, q, s, ex);
	case 6 | 2 << 8:
		return fix_chunk<6, 2>(a, q, s, ex);
	case 4 | 2 << 8:
		return fix_chunk<4, 2>(a, q, s, ex);
	case 8 | 1 << 8:
		return fix_chunk<8, 1>(a, q, s, ex);
	case 6 | 1 << 8:
		return fix_chunk<6, 1>(a, q, s, ex);
	default:
		return fix_chunk<4, 1>(a, q, s, ex);
	}
}

/*
 * Sequential tail of a batch (lane 0 of one wave): drain the re-check queue
 * in global chunk order.  Global chunk
 * indices never cross streams (a stream's chunk 0 is never queued).
 */
__device__ __forceinline__ void
drain_batch(const xa_batch_args &b)
{
	const uint32_t nq = b.ctl[XA_CTL_NQ];
	uint32_t n = 0;
	for (uint32_t i = 0; i < nq; i++)
		heap_push(b.queue, n, b.queue[i]);
	while (n > 0) {
		const uint32_t Q = heap_pop(b.queue, n);
		const uint2 s = b.e[Q - 1], gq = b.g[Q];
		if (s.x == gq.x && s.y == gq.y)
			continue;
		const uint32_t sid = b.wstream[Q / 64];
		const xa_dec_args a = batch_stream_args(b, sid);
		const uint32_t q = Q - b.streams[sid].cbase;
		uint2 ex;
		const bool met = fix_any(a, b.streams[sid].fmt, q, s, ex);
		b.g[Q] = s;
		b.sctl[sid * XA_SCTL_WORDS + XA_SCTL_TAIL]++;
		if (!met && q + 1 < a.nchunks)
			heap_push(b.queue, n, Q + 1);
	}
}

/*
 * fix_chunk for one stream of a batch, wave-uniform: the format switch does
 * not diverge, and a stream under 4 GiB of XA reads its repair windows
 * through a buffer descriptor (the descriptor must be uniform, so this
 * needs every lane of the wave on the same stream)
 */
__device__ __forceinline__ bool
fix_uniform(const xa_dec_args &a, uint32_t fmt, uint32_t q, uint2 s, uint2 &ex)
{
	const bool buf = (uint64_t)a.eblocks * ((fmt & 0xffu) * 4u + 1u) *
	    (fmt >> 8) < (1ull << 32) - 256u;
	bool met = false;
	with_format(fmt, [&](auto bc, auto cc) {
		constexpr int B = decltype(bc)::value, C = decltype(cc)::value;
		met = buf ? fix_chunk<B, C, true>(a, q, s, ex) :
		    fix_chunk<B, C, false>(a, q, s, ex);
	});
	return met;
}

/*
 * K2 over a batch.  Global wave g's 64 chunks all belong to stream
 * wstream[g], so a wave takes one global wave at a time: lane l checks
 * chunk 64g + l against its predecessor and, if they differ, repairs it in
 * place.  The stream's descriptor is wave-uniform (scalar loads), so is its
 * format, and the repair windows come through a buffer descriptor -- the
 * first version listed the mismatches of 512 chunks in LDS and gave them
 * to lanes in any order, so a wave mixed streams and formats: per-lane
 * descriptor loads, every format's path run in turn, clamped pointers
 * (C4 47 us, C5g 29 us against 18 us for one C3 stream).  The last
 * workgroup (arrival ticket) drains the cascades and publishes every
 * stream's status.
 */
__global__ __launch_bounds__(64 * XA_FIXB_WPB) void
xa_decode_fix_batch(xa_batch_args b)
{
	__shared__ uint32_t last;
	const int lane = threadIdx.x & 63;
	const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint64_t *e64 = (const uint64_t *)b.e;
	const uint64_t *g64 = (const uint64_t *)b.g;
	bool wrote = false;
	for (uint32_t gw = blockIdx.x * XA_FIXB_WPB + wv; gw < b.nwaves;
	    gw += gridDim.x * XA_FIXB_WPB) {
		const uint32_t sid = __builtin_amdgcn_readfirstlane(b.wstream[gw]);
		const xa_dec_args a = batch_stream_args(b, sid);
		const uint32_t cbase = __builtin_amdgcn_readfirstlane(b.streams[sid].cbase);
		const uint32_t fmt = __builtin_amdgcn_readfirstlane(b.streams[sid].fmt);
		const uint32_t Q = 64u * gw + (uint32_t)lane, q = Q - cbase;
		/* a stream's chunk 0 and the padding slots past its last chunk
		 * are never checked; e[Q-1] is read whatever q is (no load
		 * under a branch) */
		const uint64_t ev = __hip_atomic_load(&e64[Q > 0 ? Q - 1 : 0],
		    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		const uint64_t gv = g64[Q];
		const bool mism = q > 0 && q < a.nchunks && ev != gv;
		const uint64_t bal = __ballot(mism);
		if (bal == 0)
			continue;
		wrote = true;
		if (lane == 0)
			atomicAdd(&b.sctl[sid * XA_SCTL_WORDS + XA_SCTL_FIXED],
			    (uint32_t)__builtin_popcountll(bal));
		if (mism) {
			const uint2 s = make_uint2((uint32_t)ev, (uint32_t)(ev >> 32));
			uint2 ex;
			const bool met = fix_uniform(a, fmt, q, s, ex);
			b.g[Q] = s;
			if (!met && q + 1 < a.nchunks) {
				uint32_t i = atomicAdd(&b.ctl[XA_CTL_NQ], 1u);
				b.queue[i] = Q + 1;
			}
		}
	}
	/* arrival ticket, as in xa_decode_fix */
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	const int any = __syncthreads_or(wrote);
	if (threadIdx.x == 0) {
		if (any) {
			xa_fix_release();
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		}
		last = atomicAdd(&b.ctl[XA_CTL_TICKET], 1u) == gridDim.x - 1;
	}
	__syncthreads();
	if (!last)
		return;
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	if (threadIdx.x == 0)
		drain_batch(b);
	__syncthreads();
	/* every stream's status: up to XA_PUB streams per thread, each loaded
	 * in full before any is written, so the dependent loads (descriptor,
	 * then the last chunk's exit state) overlap across streams */
	constexpr int XA_PUB = 4;
	for (uint32_t s0 = 0; s0 < b.nstreams; s0 += 64u * XA_FIXB_WPB * XA_PUB) {
		uint32_t err[XA_PUB], fix[XA_PUB], tail[XA_PUB], nch[XA_PUB], cc[XA_PUB],
		    ww[XA_PUB];
		uint2 fin[XA_PUB];
#pragma unroll
		for (int k = 0; k < XA_PUB; k++) {
			const uint32_t sid = min(s0 + threadIdx.x + 64u * XA_FIXB_WPB * k,
			    b.nstreams - 1);
			const xa_batch_stream &d = b.streams[sid];
			const uint32_t *sc = b.sctl + sid * XA_SCTL_WORDS;
			nch[k] = d.nchunks;
			cc[k] = d.C;
			ww[k] = d.nlong ? d.Wlong + d.dlong : b.W;
			fin[k] = b.e[d.cbase + d.nchunks - 1];
			err[k] = sc[XA_SCTL_ERR];
			fix[k] = sc[XA_SCTL_FIXED];
			tail[k] = sc[XA_SCTL_TAIL];
		}
#pragma unroll
		for (int k = 0; k < XA_PUB; k++) {
			const uint32_t sid = s0 + threadIdx.x + 64u * XA_FIXB_WPB * k;
			if (sid >= b.nstreams)
				continue;
			uint32_t *sc = b.sctl + sid * XA_SCTL_WORDS;
			uint32_t *st = b.status + sid * XA_ST_WORDS;
			st[XA_ST_ERR] = err[k];
			st[XA_ST_STATE_L] = fin[k].x;
			st[XA_ST_STATE_R] = fin[k].y;
			st[XA_ST_FIXED] = fix[k];
			st[XA_ST_TAIL] = tail[k];
			st[XA_ST_CHUNKS] = nch[k];
			st[XA_ST_C] = cc[k];
			st[XA_ST_W] = ww[k];
			sc[XA_SCTL_ERR] = 0xffffffffu;
			sc[XA_SCTL_FIXED] = 0;
			sc[XA_SCTL_TAIL] = 0;
		}
	}
	if (threadIdx.x == 0) {
		b.ctl[XA_CTL_NQ] = 0;
		b.ctl[XA_CTL_TICKET] = 0;
	}
}

hipError_t
xa_decode_batch_launch(const xa_batch_args &b, hipStream_t st, hipEvent_t ev0,
    hipEvent_t ev1)
{
	const unsigned grid = (b.nwaves + XA_SPEC_WPB - 1) / XA_SPEC_WPB;
	/* K2: a wave per global wave, XA_FIXB_WPB per workgroup, at most
	 * XA_FIXB_MAXWG workgroups */
	unsigned grid2 = (b.nwaves + XA_FIXB_WPB - 1) / XA_FIXB_WPB;
	if (grid2 > XA_FIXB_MAXWG)
		grid2 = XA_FIXB_MAXWG;
	if (ev0 != NULL)
		(void)hipEventRecord(ev0, st);
	hipLaunchKernelGGL((xa_decode_spec_batch<128, true>), dim3(grid),
	    dim3(64 * XA_SPEC_WPB), 0, st, b);
	if (ev1 != NULL)
		(void)hipEventRecord(ev1, st);
	hipLaunchKernelGGL(xa_decode_fix_batch, dim3(grid2), dim3(64 * XA_FIXB_WPB), 0,
	    st, b);
	return hipGetLastError();
}
