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
 *                     together -- then decodes its chunk, emitting PCM.
 *                     Chunk 0 starts from the true caller state and needs
 *                     no warm-up.  Chunk q is correct iff chunk q-1 is and
 *                     its entry state equals q-1's exit.  Each wave then
 *                     settles its own boundaries: its last lane publishes
 *                     its exit for the next wave (a tagged record), every
 *                     lane compares its entry with the exit of the chunk
 *                     before it (a lane shuffle; lane 0 reads the previous
 *                     wave's record), and each mismatching chunk is
 *                     re-decoded by its own lane from the true entry, block
 *                     by block, until its block-end state meets the stored
 *                     trajectory (everything after is then unchanged).  A
 *                     chunk that never meets it, or a record that does not
 *                     come in time, queues a chunk for K2.  The repairs run
 *                     on the CU that wrote the PCM, beside the waves still
 *                     decoding, not after the whole grid.
 *  K2 xa_decode_tail  one workgroup: drains that queue in chunk order with
 *                     one thread, so a cascade through several chunks is
 *                     repaired exactly, and publishes the status.
 *
 * By induction from chunk 0 every chunk ends up decoded from its true start
 * state: the output is bit-exact for any input; speculation only sets the
 * cost.
 *
 * Memory (K1).  A lane's input for a "super-step" (two groups of 4 channel
 * blocks) is one contiguous run of the stream; the runs of half a wave land
 * together in one LDS buffer by LDS-DMA, every DMA instruction filling
 * 1 KiB of LDS, and each lane copies its run to VGPRs.  The next
 * super-step's run lands while this one decodes.  The PCM of each eblock is
 * staged in LDS, 128 B per lane, and stored so that each instruction covers
 * 8 whole lines.
 * Predictor: stereo runs both channels as the two halves of packed-f32
 * instructions (xa_step_lr), mono a single f32 chain (xa_step_f); both are
 * exact (xa_common.h).
 */
#include "xa_kern.h"

#ifndef XA_SPEC_WPB
#define XA_SPEC_WPB 4		/* waves per K1 workgroup */
#endif
#define XA_SPEC_CPW (64 * XA_SPEC_WPB)	/* chunks per K1 workgroup */
#ifndef XA_FIX_PF
#define XA_FIX_PF 4		/* repair windows in flight per lane */
#endif
#define XA_TAIL_THREADS 256	/* K2 workgroup size */

static_assert(XA_SCTL_FIXED == XA_CTL_FIXED && XA_SCTL_ERR == XA_CTL_ERR,
    "a batch stream's control words double as xa_dec_args::ctl");

/* bytes of PCM per lane per store phase: one stereo eblock, two mono */
#define XA_LB 128
#define XA_NST 16	/* store instructions per group (G * OB / 16) */

/*
 * The wave's output stage: where lane j's XA_LB-byte line sits, and where
 * each of its eight 16-B pieces sits in it.  Banking (MI355X_MICROARCH.md
 * §LDS): ds_write_b128 serves 8 contiguous lanes a cycle on 32 banks,
 * ds_read_b128 16 lanes a cycle on 64 banks in the non-contiguous groups
 * {0-3,12-15,20-27} {4-11,16-19,28-31} and the same +32.
 *   Lanes write the same piece of their own lines at once, so the 8 line
 *   starts of a write group must be distinct mod 128 B.  Lines 2m and
 *   2m+1 share a 272-B block: 2m at 272m, 2m+1 at 272m + 64, pieces 4-7
 *   of a line 64 B further than 0-3 (ost_piece), so the pair interleaves
 *   in 64-B halves and the block's 16-B slot index mod 8 is (m + 4(j&1))
 *   mod 8: distinct over 8 consecutive lines.
 *   The stores read 8 lines (4 blocks) a pass; each 4-lane quad reads one
 *   half line, and ost_quad gives each read group the four halves of one
 *   block -- 16 distinct slots mod 256 B.
 * Both are conflict-free (tools/lds_banks.py); the round-5 pitch of
 * 128 B + 16 B per pair conflicted 2-way on every write, the round-4 pitch
 * of 144 B on the reads.  The stage is 64 lines in 32 blocks, 8704 B, as
 * before.
 */
__host__ __device__ constexpr int
ost_line(int j)
{
	return (j >> 1) * (2 * XA_LB + 16) + (j & 1) * (XA_LB / 2);
}
__host__ __device__ constexpr int
ost_piece(int p)
{
	return 16 * (p + (p & 4));
}
/* quad q (lanes 4q..4q+3) of a store pass reads half (c & 1) of line c >> 1
 * of the pass, c = nibble q */
__device__ __forceinline__ void
ost_quad(int lane, int &jj, int &pc)
{
	const uint32_t c = (uint32_t)(0xfbae9dc873261540ull >> (4 * (lane >> 2))) & 15u;
	jj = (int)(c >> 1);
	pc = (int)(c & 1u) * 4 + (lane & 3);
}

/* one 16-B piece of PCM, streamed out: non-temporal (the line stays in the
 * XCD's L2 until evicted), or with XA_PCM_SC1 system-coherent write-through
 * (MI355X_MICROARCH.md: sc1 stores leave L2 at once and drop the line) */
__device__ __forceinline__ void
pcm_store(uint8_t *p, const u32x4a v)
{
#ifdef XA_PCM_SC1
	asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) :
	    "memory");
#else
	__builtin_nontemporal_store(v, (u32x4a *)p);
#endif
}

/*
 * Store the wave's staged XA_LB-byte lines: line j belongs to chunk
 * wchunk0 + j (whose PCM starts at wstart_b + j * chunk_bytes) and goes to
 * byte `rel_off` of that chunk's PCM.  Pass i stores lines 8i .. 8i+7,
 * lane l the piece of them ost_quad names.  Wave-uniform fast path when
 * every line is whole; a predicated copy of it when the stream ends inside
 * the wave on a 16-B boundary; otherwise (a cut last block) per-piece
 * bounds and a 2-byte tail.  Stores are non-temporal (measured best for every format, DESIGN.md
 * §3).
 */
__device__ __forceinline__ void
store_lines(const xa_dec_args &a, const uint8_t *obuf, int lane,
    uint32_t wchunk0, uint64_t wstart_b, uint32_t chunk_bytes, uint32_t rel_off,
    bool wave_full, bool clean, uint8_t *gbase, const uint8_t *lbase)
{
	constexpr int P = XA_LB / 16, LPI = 64 / P, LSTEP = ost_line(LPI);
	static_assert(ost_line(LPI + 1) - ost_line(1) == LSTEP &&
	    ost_line(LPI + 2) - ost_line(2) == LSTEP, "stage stride");
	if (wave_full) {
		uint8_t *gp = gbase + rel_off;
		const uint64_t istride = (uint64_t)LPI * chunk_bytes;
#pragma unroll
		for (int i = 0; i < P; i++) {
			const u32x4a v = *(const u32x4a *)(lbase + i * LSTEP);
			pcm_store(gp + i * istride, v);
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
			const u32x4a v = *(const u32x4a *)(lbase + i * LSTEP);
			uint8_t *q = gp + i * istride;
			if (q + 16 <= end)
				pcm_store(q, v);
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
		int jj, pc;
		ost_quad(lane, jj, pc);
		const int j = i * LPI + jj;
		const uint32_t cj = wc + (uint32_t)j;
		const uint64_t off = wsb + (uint64_t)j * cb + ro + (uint64_t)pc * 16u;
		if (cj >= nch)
			continue;
		const uint8_t *from = obuf + ost_line(j) + ost_piece(pc);
		/* (off < lim first, so that no bound can wrap) */
		if (off >= lim)
			continue;
		if (lim - off >= 16u) {
			*(u32x4a *)(dst + off) = *(const u32x4a *)from;
		} else {
			for (uint64_t k = 0; off + k < lim; k += 2)
				*(uint16_t *)(dst + off + k) =
				    *(const uint16_t *)(from + k);
		}
	}
}

template <int BITS, int CH> struct geo2 {
	typedef geo<BITS, CH> g;
	static constexpr int RD = 2 * g::GDW;			/* dwords per run */
	static constexpr int SLOT = (RD * 4 + 15) / 16 * 16;	/* LDS bytes per run */
	static constexpr int NPR = SLOT / 16;			/* 16-B pieces per run */
	static constexpr int NI = (32 * NPR + 63) / 64;		/* DMA instructions per half */
	static constexpr int LAST = 32 * NPR - 64 * (NI - 1);	/* lanes of the last one */
	static constexpr int HALF = 32 * SLOT;
};

/* one wave's LDS: the half-wave landing buffer, then the output stage */
template <int BITS, int CH> struct spec_lds2 {
	static constexpr int REGION = geo2<BITS, CH>::HALF + ost_line(64);
	static_assert(REGION >= 64 * 8, "the exit exchange needs 8 B per lane");
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
#ifdef XA_DBG_LINE_RUNS
	/* the diagnostic's own footprint: runs at whole-line strides reach
	 * further than the real ones */
	const bool inside = e_first >= 0 && (int64_t)(((size_t)c0 * g::EBSZ) &
	    ~(size_t)127) + (rel + (int64_t)a.W) / (2 * g::G) * 256 +
	    32 * (int64_t)((Cw * g::EBSZ + 127u) & ~127u) <=
	    (int64_t)a.eblocks * g::EBSZ;
#else
	const int64_t e_end = c0 + 31 * (int64_t)Cw + rel + 2 * g::G;
	const bool inside = e_first >= 0 && e_end * g::EBSZ +
	    (g2::SLOT - 4 * g2::RD) <= (int64_t)a.eblocks * g::EBSZ;
#endif
	if (inside) {
#ifdef XA_DBG_LINE_RUNS
		/* diagnostic build only (wrong output): every run is two whole
		 * 128-B lines, runs of a lane back to back (no line is fetched
		 * twice), lane bases on lines; the same DMA and decode work */
		const uint8_t *base = a.src + (((size_t)c0 * g::EBSZ) & ~(size_t)127) +
		    (size_t)(rel + (int64_t)a.W) / (2 * g::G) * 256;
#else
		const uint8_t *base = a.src + (size_t)e_first * g::EBSZ;
#endif
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

/* ------------------------------------------------------------------ */
/* repair                                                               */

/*
 * Re-decode chunk q from the state s (s.x: channel 0, s.y: channel 1),
 * rewriting its PCM, on one lane: the eblock goes through K1's own
 * decode_eblock (stereo: both channels in one packed-f32 instruction stream,
 * 11 VALU per frame, with the output frame packed by the step itself; mono:
 * the f32 chain), so repaired PCM is K1's arithmetic bit for bit.  Stops
 * once a block-end state equals the stored trajectory (frames 30/31 of the
 * old PCM) in every channel: nothing after it can change.  Returns true if
 * it met the trajectory; otherwise returns the chunk's new exit state in
 * `exit` (the caller records it).
 *
 * The repair is one serial chain per chunk, so its time is its instruction
 * count (~11 VALU per frame, ~1 us per block alone).
 *
 * No load sits under a branch (hipcc drains vmcnt(0) right after such
 * loads): the windows and old end states of the blocks XA_FIX_PF ahead are
 * fetched every iteration with clamped addresses.  The windows come through
 * a buffer descriptor whose base is eblock `bb` of the stream (bb <= the
 * chunk's first eblock, the same for every active lane: the wave's first
 * eblock in K1, the chunk's own in the one-thread tail) and whose range
 * ends with the stream, so its range check returns 0 past the end instead
 * of per-dword 64-bit clamps.  The planner keeps a wave's span of XA under
 * 4 GiB (xa_gpu.hip), so every offset fits the descriptor's 32 bits.
 */
template <int BITS, int CH>
__device__ __forceinline__ bool
fix_chunk(const xa_dec_args &a, uint32_t q, uint2 s, uint2 &exit, int64_t bb)
{
	typedef geo<BITS, CH> g;
	constexpr int EBSZ = g::EBSZ, OB = g::OB;
	constexpr int WN = (EBSZ + 3) / 4;	/* dwords of one eblock */
	int32_t p0[CH], p1[CH];
	xa_unpack_state(s.x, p0[0], p1[0]);
	if (CH == 2)
		xa_unpack_state(s.y, p0[CH - 1], p1[CH - 1]);
	const int64_t eblocks = a.eblocks;
	const int64_t b0 = (int64_t)q * a.C;
	int64_t b1 = b0 + a.C;
	if (b1 > eblocks)
		b1 = eblocks;
	/* q >= 1, so the stream has whole blocks (nfull >= b0 >= 16) */
	const int64_t nfull = (int64_t)(a.pcm_bytes / OB);

	/* the descriptor: base at eblock bb's dword, range to the stream's end
	 * (at most 2^32 - 256 bytes) */
	const uint64_t base_b = ((uint64_t)bb * EBSZ) & ~(uint64_t)3;
	const uint64_t span = ((uint64_t)eblocks * EBSZ + 3u) / 4u * 4u - base_b;
	__amdgpu_buffer_rsrc_t rs;
	{
		const uint64_t sp = (uint64_t)a.src + base_b;
		const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)sp);
		const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(sp >> 32));
		const uint32_t nb = __builtin_amdgcn_readfirstlane((uint32_t)min(span,
		    (uint64_t)0xffffff00u));
		rs = __builtin_amdgcn_make_buffer_rsrc(
		    (void *)(((uint64_t)hi << 32) | lo), 0, (int)nb, 0x00020000);
	}
	/* the WN + 1 dwords holding eblock b */
	auto fetch = [&](uint32_t *r, int64_t b) {
		/* dwords 0 .. NIN-1 hold only bytes of eblock b (whatever its
		 * alignment), so 16-B loads there never straddle the range
		 * check; the rest one dword at a time */
		constexpr int NIN = (EBSZ - 1) / 4 + 1, N4 = NIN / 4;
		const uint32_t o = (uint32_t)((((uint64_t)b * EBSZ) & ~(uint64_t)3) -
		    base_b);
#pragma unroll
		for (int i = 0; i < N4; i++) {
			const u32x4a v = __builtin_bit_cast(u32x4a,
			    __builtin_amdgcn_raw_buffer_load_b128(rs,
			    (int)(o + 16u * i), 0, 0));
			r[4 * i] = v.x;
			r[4 * i + 1] = v.y;
			r[4 * i + 2] = v.z;
			r[4 * i + 3] = v.w;
		}
#pragma unroll
		for (int i = 4 * N4; i <= WN; i++)
			r[i] = __builtin_amdgcn_raw_buffer_load_b32(rs,
			    (int)(o + 4u * i), 0, 0);
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
	return false;
}

/*
 * The exit record a wave leaves for the next one: lane 63's exit state as
 * two 8-B granules {state, launch tag}, each written by one agent-scope
 * atomic store and read by agent-scope atomic loads (write-through and
 * L1-bypassing: the placement-independent granule hand-off of
 * MI355X_MICROARCH.md, which needs no fence), so a reader sees either this
 * launch's record or one it recognises as not yet written (a torn read
 * fails the tag of one half).  Nothing else passes between waves: each wave
 * repairs only the PCM it wrote itself.
 */
__device__ __forceinline__ void
put_exit(uint4 *rec, uint2 ex, uint32_t tag)
{
	uint64_t *p = (uint64_t *)rec;
	__hip_atomic_store(p, (uint64_t)ex.x | (uint64_t)tag << 32,
	    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	__hip_atomic_store(p + 1, (uint64_t)ex.y | (uint64_t)tag << 32,
	    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool
get_exit(const uint4 *rec, uint32_t tag, uint2 &ex)
{
	const uint64_t *p = (const uint64_t *)rec;
	const uint64_t lo = __hip_atomic_load(p, __ATOMIC_RELAXED,
	    __HIP_MEMORY_SCOPE_AGENT);
	const uint64_t hi = __hip_atomic_load(p + 1, __ATOMIC_RELAXED,
	    __HIP_MEMORY_SCOPE_AGENT);
	ex = make_uint2((uint32_t)lo, (uint32_t)hi);
	return (uint32_t)(lo >> 32) == tag && (uint32_t)(hi >> 32) == tag;
}

/* queue stream chunk q for K2's in-order re-check; past the queue's
 * capacity (only a workspace left inconsistent by a failed launch gets
 * there) K2 re-checks every boundary instead, so nothing is dropped */
__device__ __forceinline__ void
enqueue(const xa_dec_args &a, uint32_t q)
{
	const uint32_t j = atomicAdd(a.nq, 1u);
	if (j < a.qcap)
		a.queue[j] = a.qbase + q;
	else
		atomicOr(a.ovf, 1u);
}

/*
 * After K1's main loop: the wave settles the boundaries of its 64 chunks.
 * Lane l holds stream chunk q = wchunk0 + l with entry state gs and exit
 * state ex.  Chunk q is correct iff q-1 is and gs equals q-1's exit: lane
 * l-1's (a shuffle), or for lane 0 the previous wave's record, which lane
 * 63 of that wave published right after its main loop.  Every mismatching
 * lane re-decodes its own chunk from that exit (fix_chunk, one serial chain
 * per lane, all of the wave's repairs side by side); a repair that does not
 * meet the stored trajectory changes q's exit and queues q+1 for K2, so
 * checking against the speculative exits is exact.  If the previous wave's
 * record is not there at once, the wave first does its other repairs, then
 * lane 0 polls for up to `a.spin` ticks (an exit condition every wave
 * reaches: nothing here waits on a workgroup that might not be resident);
 * a record that does not come queues q itself for K2.  Finally each lane
 * records the entry it was decoded from and its exit (g[q], e[q]) for K2.
 */
template <int BITS, int CH>
__device__ __forceinline__ void
settle_wave(const xa_dec_args &a, int lane, uint32_t wchunk0, uint2 gs, uint2 ex)
{
	const uint32_t q = wchunk0 + (uint32_t)lane, n = a.nchunks;
	const bool live = q < n;
	const uint32_t wl = wchunk0 / 64u;	/* the wave within its stream */
	const bool norec = (a.flags & XA_F_NORECORD) != 0u;
	if (lane == 63 && q + 1u < n && !norec)
		put_exit(&a.exits[wl], ex, a.tag);
	uint2 s = make_uint2(__shfl_up(ex.x, 1), __shfl_up(ex.y, 1));
	bool wait = live && lane == 0 && wchunk0 > 0;
	bool chk = live && lane > 0;
	if (wait && norec) {
		enqueue(a, q);
		wait = false;
	}
	if (wait && get_exit(&a.exits[wl - 1], a.tag, s)) {
		wait = false;
		chk = true;
	}
	/* the wave's own PCM stores are complete before repairs read them */
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	uint2 g = gs, e = ex;
	bool fixed = false;
#pragma nounroll
	for (int round = 0; round < 2; round++) {
		if (round == 1) {
			if (__ballot(wait) == 0)
				break;
			if (wait) {
				const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
				bool got;
				while (!(got = get_exit(&a.exits[wl - 1], a.tag, s)) &&
				    __builtin_amdgcn_s_memrealtime() - t0 < a.spin)
					__builtin_amdgcn_s_sleep(2);
				if (got)
					chk = true;
				else
					enqueue(a, q);
			}
		}
		const bool fix = chk && (s.x != gs.x || s.y != gs.y);
		chk = false;
		if (__ballot(fix) == 0)
			continue;
		if (fix) {
			uint2 nx;
			const bool met = fix_chunk<BITS, CH>(a, q, s, nx,
			    (int64_t)wchunk0 * a.C);
			g = s;
			fixed = true;
			if (!met) {
				e = nx;
				if (q + 1u < n)
					enqueue(a, q + 1u);
			}
		}
	}
	const uint64_t nf = __ballot(fixed);
	if (nf != 0 && lane == 0)
		atomicAdd(&a.ctl[XA_CTL_FIXED], (uint32_t)__builtin_popcountll(nf));
	if (live) {
		a.g[q] = g;
		a.e[q] = e;
	}
}

/* ------------------------------------------------------------------ */
/* K1                                                                   */

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
 * staged in a separate region.  Leaves the lane's entry state (gs) and
 * exit state (ex), packed.
 */
template <int BITS, int CH>
__device__ __forceinline__ void
spec_wave2(const xa_dec_args &a, uint8_t *region, const uint32_t wchunk0,
    const uint32_t pace_every, uint2 &gs, uint2 &ex)
{
	typedef geo<BITS, CH> g;
	typedef geo2<BITS, CH> g2;
	constexpr int G = g::G, OB = g::OB, EBSZ = g::EBSZ, GDW = g::GDW;
	constexpr int RD = g2::RD, LB = XA_LB;
	static_assert(G * OB / 16 == XA_NST, "store count per group");

	const int lane = threadIdx.x & 63;
	uint8_t *land = region, *ost = region + g2::HALF;
	const int64_t eblocks = a.eblocks;
	const uint32_t Cw = a.C;
	const int64_t wstart = (int64_t)wchunk0 * Cw;
	const int64_t b0 = wstart + (int64_t)lane * Cw;
	const int W = (int)a.W;
	/* super-steps: NW of warm-up, then NC of the chunk (W and Cw are
	 * multiples of 2G, the host plans them so) */
	const int NW = W / (2 * G), NS = NW + (int)Cw / (2 * G);

	uint32_t voff[g2::NI];
#pragma unroll
	for (int i = 0; i < g2::NI; i++) {
		const int k = i * 64 + lane;
#ifdef XA_DBG_LINE_RUNS
		voff[i] = (uint32_t)(k / g2::NPR) * ((Cw * EBSZ + 127u) & ~127u) +
		    (uint32_t)min(k % g2::NPR, 15) * 16u;
#else
		voff[i] = (uint32_t)(k / g2::NPR) * Cw * EBSZ +
		    (uint32_t)(k % g2::NPR) * 16u;
#endif
	}

	int32_t p0[CH], p1[CH];
#pragma unroll
	for (int c = 0; c < CH; c++) {
		if (b0 - W <= 0)	/* the stream start: the caller's state */
			xa_unpack_state(a.init_dev != nullptr ?
			    a.init_dev[XA_ST_STATE_L + c] : a.init[c], p0[c], p1[c]);
		else
			p0[c] = p1[c] = 0;
	}
	uint32_t gst[2] = { 0u, 0u };

	const uint32_t chunk_bytes = Cw * OB;
	const uint64_t wstart_b = (uint64_t)wstart * OB;
	int sj, sp;
	ost_quad(lane, sj, sp);
	uint8_t *gbase = a.dst + wstart_b + (uint64_t)sj * chunk_bytes + sp * 16;
	const uint8_t *lbase = ost + ost_line(sj) + ost_piece(sp);
	uint8_t *line = ost + ost_line(lane);
	const uint64_t full_blocks = a.pcm_bytes / OB;
	const bool wave_full = wchunk0 + 63u < a.nchunks &&
	    (uint64_t)(wstart + 64 * (int64_t)Cw) <= full_blocks;
	const bool clean = (a.pcm_bytes & 15u) == 0;
	auto none = [](int) {};

	/* copy this lane's run out of the landing buffer (half h only) */
	auto take = [&](int h, uint32_t *dst) {
		if ((lane >> 5) == h) {
			/* whole 16-B reads (left to itself the compiler split
			 * one of the two buffers into ds_read2_b32 pairs, 4-way
			 * bank conflicts at the 272-B run stride) */
			const uint8_t *m = land + (lane & 31) * g2::SLOT;
#pragma unroll
			for (int i = 0; i + 4 <= RD; i += 4) {
				const u32x4a v = *(const u32x4a *)(m + 4 * i);
				dst[i] = v[0];
				dst[i + 1] = v[1];
				dst[i + 2] = v[2];
				dst[i + 3] = v[3];
			}
#pragma unroll
			for (int i = RD & ~3; i < RD; i++)
				dst[i] = ((const uint32_t *)m)[i];
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	};
	auto rel_of = [&](int S) -> int64_t { return (int64_t)S * 2 * G - W; };
	/* wait for the DMA issued just before decoding group gi: only that
	 * group's stores are younger, when it stored on the fast path */
	auto wait_after = [&](int gi) {
		if (gi >= 2 * NW && wave_full)
			asm volatile("s_waitcnt vmcnt(%0)" :: "n"(XA_NST) : "memory");
		else
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
				store_lines(a, ost, lane, wchunk0, wstart_b,
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
#ifdef XA_DBG_LINE_RUNS	/* (its garbage profiles would all contend here) */
			bad = 0;
#endif
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
	 * next requests sooner (C3 spec -1.3 %, C2 -1.6 %) */
	auto prio = [](auto pc) {
		__builtin_amdgcn_s_setprio(decltype(pc)::value);
	};
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
	/* one super-step from run `cur`, landing the next one into `nxt` */
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
	gs = make_uint2(gst[0], gst[1]);
	ex = make_uint2(xa_pack_state(p0[0], p1[0]),
	    CH == 2 ? xa_pack_state(p0[CH - 1], p1[CH - 1]) : 0u);
}

/* K1 for one stream: wave w of the grid takes chunks 64w .. 64w+63 and
 * settles their boundaries */
template <int BITS, int CH>
__global__ __launch_bounds__(XA_SPEC_CPW, 8 / XA_SPEC_WPB) void
xa_decode_spec(xa_dec_args a)
{
	/* the wave index is wave-uniform; say so, so that LDS bases and the
	 * DMA source base live in SGPRs */
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	typedef spec_lds2<BITS, CH> L;
	__shared__ __attribute__((aligned(16))) uint8_t
	    lds[XA_SPEC_WPB * L::REGION];
	const uint32_t wchunk0 = blockIdx.x * XA_SPEC_CPW + wv * 64u;
	uint2 gs, ex;
	spec_wave2<BITS, CH>(a, lds + wv * L::REGION, wchunk0, a.pace, gs, ex);
#ifdef XA_DBG_LINE_RUNS
	return;		/* diagnostic build: its PCM is garbage */
#endif
	settle_wave<BITS, CH>(a, lane, wchunk0, gs, ex);
}

/* ------------------------------------------------------------------ */
/* K2: the sequential tail                                              */

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
 * The sequential tail (thread 0): drain the re-check queue in chunk order
 * (a heap, so even a pathological cascade costs O(n log n) bookkeeping),
 * then publish the status words and reset the control words.  Entries
 * outside [1, nchunks) -- stale ones, from a workspace a failed launch left
 * behind -- are skipped, so nothing is read out of range.
 */
template <int BITS, int CH>
__device__ __forceinline__ void
drain_tail(const xa_dec_args &a)
{
	const uint32_t nq = min(*a.nq, a.qcap), nc = a.nchunks;
	uint32_t n = 0, tail = 0;
	for (uint32_t i = 0; i < nq; i++) {
		const uint32_t q = a.queue[i];
		if (q >= 1u && q < nc)
			heap_push(a.queue, n, q);
	}
	while (n > 0) {
		const uint32_t q = heap_pop(a.queue, n);
		const uint2 s = a.e[q - 1], gq = a.g[q];
		if (s.x == gq.x && s.y == gq.y)
			continue;
		tail++;
		uint2 ex;
		const bool met = fix_chunk<BITS, CH>(a, q, s, ex, (int64_t)q * a.C);
		a.g[q] = s;
		if (!met) {
			a.e[q] = ex;
			if (q + 1 < nc)
				heap_push(a.queue, n, q + 1);
		}
	}
	const uint2 fin = a.e[nc - 1];
	a.status[XA_ST_ERR] = a.ctl[XA_CTL_ERR];
	a.status[XA_ST_STATE_L] = fin.x;
	a.status[XA_ST_STATE_R] = fin.y;
	a.status[XA_ST_FIXED] = a.ctl[XA_CTL_FIXED];
	a.status[XA_ST_TAIL] = tail;
	a.status[XA_ST_CHUNKS] = nc;
	a.status[XA_ST_C] = a.C;
	a.status[XA_ST_W] = a.W;
	a.ctl[XA_CTL_ERR] = 0xffffffffu;
	a.ctl[XA_CTL_NQ] = 0;
	a.ctl[XA_CTL_FIXED] = 0;
	a.ctl[XA_CTL_OVF] = 0;
}

/*
 * After a queue overflow (XA_CTL_OVF) the queue is rebuilt from scratch:
 * every boundary of [first, end) (global chunk indices) whose entry state
 * differs from its predecessor's exit, found by the whole workgroup, written
 * as queue entries; skip(Q) drops indices that are no boundary (a batch
 * stream's chunk 0, padding).  Returns on every thread; thread 0 then holds
 * the new length in *nq.
 */
template <typename F>
__device__ __forceinline__ void
rebuild_queue(const uint2 *e, const uint2 *g, uint32_t *queue, uint32_t *nq,
    uint32_t first, uint32_t end, F &&skip)
{
	__shared__ uint32_t cnt;
	if (threadIdx.x == 0)
		cnt = 0;
	__syncthreads();
	for (uint32_t Q = first + threadIdx.x; Q < end; Q += blockDim.x) {
		if (skip(Q))
			continue;
		const uint2 s = e[Q - 1], gq = g[Q];
		if (s.x != gq.x || s.y != gq.y)
			queue[atomicAdd(&cnt, 1u)] = Q;
	}
	__syncthreads();
	if (threadIdx.x == 0)
		*nq = cnt;
	__syncthreads();
}

/*
 * Before the one-thread drain: the whole workgroup drops the queued entries
 * that need no repair (keep(Q) false: out of range, no boundary, or entry
 * state already equal to the predecessor's exit), so the drain's serial
 * loop only sees real mismatches.  Dropping an entry whose states match is
 * safe: if a repair earlier in the drain changes that predecessor's exit,
 * the cascade queues the entry again.  Up to XA_TAIL_KEEP survivors are
 * compacted to the front of the queue; past that the queue is left whole
 * and the drain checks every entry itself.  This keeps the tail cheap when
 * many waves left their first boundary to it (their records came late:
 * other kernels holding the GPU).
 */
#define XA_TAIL_KEEP 4096

template <typename F>
__device__ __forceinline__ void
filter_queue(uint32_t *queue, uint32_t *nq, uint32_t qcap, F &&keep)
{
	__shared__ uint32_t cnt;
	__shared__ uint32_t kept[XA_TAIL_KEEP];
	if (threadIdx.x == 0)
		cnt = 0;
	__syncthreads();
	const uint32_t n = min(*nq, qcap);
	for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
		const uint32_t Q = queue[i];
		if (keep(Q)) {
			const uint32_t j = atomicAdd(&cnt, 1u);
			if (j < XA_TAIL_KEEP)
				kept[j] = Q;
		}
	}
	__syncthreads();
	const uint32_t c = cnt;
	if (c <= XA_TAIL_KEEP) {
		for (uint32_t i = threadIdx.x; i < c; i += blockDim.x)
			queue[i] = kept[i];
		__syncthreads();
		if (threadIdx.x == 0)
			*nq = c;
	}
	__syncthreads();
}

/* the entry state of chunk Q differs from its predecessor's exit */
__device__ __forceinline__ bool
differs(const uint2 *e, const uint2 *g, uint32_t Q)
{
	const uint2 s = e[Q - 1], gq = g[Q];
	return s.x != gq.x || s.y != gq.y;
}

/*
 * K2 for one stream: one workgroup.  Everything K1 could not settle itself
 * is in the queue (cascades out of a chunk, boundaries whose record did not
 * come in time); thread 0 re-checks it in chunk order and publishes the
 * status.  Its cost is a launch and, almost always, an empty queue.
 */
template <int BITS, int CH>
__global__ __launch_bounds__(XA_TAIL_THREADS) void
xa_decode_tail(xa_dec_args a)
{
	if (*a.ovf != 0u)
		rebuild_queue(a.e, a.g, a.queue, a.nq, 1u, a.nchunks,
		    [](uint32_t) { return false; });
	else
		filter_queue(a.queue, a.nq, a.qcap, [&](uint32_t q) {
			return q >= 1u && q < a.nchunks && differs(a.e, a.g, q);
		});
	if (threadIdx.x == 0)
		drain_tail<BITS, CH>(a);
}

/* ------------------------------------------------------------------ */

/* the record tag of a launch: process-wide, never 0 */
static uint32_t
next_tag(void)
{
	static uint32_t t;
	uint32_t v;
	do
		v = __atomic_add_fetch(&t, 1u, __ATOMIC_RELAXED);
	while (v == 0u);
	return v;
}

template <int BITS, int CH>
static hipError_t
launch(const xa_dec_args &a0, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1)
{
	xa_dec_args a = a0;
	a.tag = next_tag();
	const unsigned grid = (a.nchunks + XA_SPEC_CPW - 1) / XA_SPEC_CPW;
	if (ev0 != NULL)
		(void)hipEventRecord(ev0, st);
	hipLaunchKernelGGL((xa_decode_spec<BITS, CH>), dim3(grid),
	    dim3(XA_SPEC_CPW), 0, st, a);
	if (ev1 != NULL)
		(void)hipEventRecord(ev1, st);
#ifdef XA_DBG_LINE_RUNS
	return hipGetLastError();	/* its PCM is garbage: nothing to verify */
#endif
	hipLaunchKernelGGL((xa_decode_tail<BITS, CH>), dim3(1),
	    dim3(XA_TAIL_THREADS), 0, st, a);
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
	a.W = b.W;
	a.pace = 0;	/* the batch kernel decides per workgroup */
	a.init[0] = d.init[0];
	a.init[1] = d.init[1];
	a.init_dev = nullptr;
	a.g = b.g + d.cbase;
	a.e = b.e + d.cbase;
	a.queue = b.queue;
	a.nq = &b.ctl[XA_CTL_NQ];
	a.qcap = 2u * 64u * b.nwaves;
	a.qbase = d.cbase;
	a.ovf = &b.ctl[XA_CTL_OVF];
	a.exits = b.exits + d.cbase / 64u;
	a.tag = b.tag;
	a.spin = b.spin;
	a.flags = b.flags;
	a.ctl = b.sctl + sid * XA_SCTL_WORDS;	/* ERR and FIXED line up */
	a.status = b.status + sid * XA_ST_WORDS;
	return a;
}

constexpr int
xa_max(int x, int y)
{
	return x > y ? x : y;
}

struct batch_lds {
	/* one region per wave (landing buffer + output stage), the
	 * largest over the formats */
	static constexpr int REGION = xa_max(xa_max(xa_max(
	    spec_lds2<8, 2>::REGION, spec_lds2<8, 1>::REGION),
	    xa_max(spec_lds2<6, 2>::REGION, spec_lds2<6, 1>::REGION)),
	    xa_max(spec_lds2<4, 2>::REGION, spec_lds2<4, 1>::REGION));
};

/*
 * K1 over a batch: wave w decodes 64 chunks of stream wstream[w] with that
 * stream's format (wave-uniform dispatch, no divergence), then settles
 * their boundaries as xa_decode_spec does (the wave before it belongs to
 * the same stream unless this wave starts the stream; queue entries are
 * global chunk indices).
 */
__global__ __launch_bounds__(XA_SPEC_CPW, 8 / XA_SPEC_WPB) void
xa_decode_spec_batch(xa_batch_args b)
{
	__shared__ __attribute__((aligned(16))) uint8_t
	    lds[XA_SPEC_WPB * batch_lds::REGION];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	const uint32_t w = blockIdx.x * XA_SPEC_WPB + wv;
	/* lockstep (spec_wave2's pacing) only when all the workgroup's waves
	 * exist and run the same number of super-steps: same chunk length and
	 * channel count */
	const uint32_t w0 = blockIdx.x * XA_SPEC_WPB;
	bool lockstep = b.pace != 0u && w0 + XA_SPEC_WPB <= b.nwaves;
	if (lockstep) {
		auto shape = [&](uint32_t wk) {
			const xa_batch_stream &d = b.streams[b.wstream[wk]];
			return (b.W + d.C) | (d.fmt >> 8) << 24;
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
	uint8_t *region = lds + wv * batch_lds::REGION;
	with_format(fmt, [&](auto bc, auto cc) {
		constexpr int BITS = decltype(bc)::value, CH = decltype(cc)::value;
		uint2 gs, ex;
		spec_wave2<BITS, CH>(a, region, wchunk0, lockstep ? b.pace : 0u,
		    gs, ex);
		settle_wave<BITS, CH>(a, lane, wchunk0, gs, ex);
	});
}

/* fix_chunk in a stream's format, for the one-thread tail (windows based at
 * the chunk itself) */
__device__ __forceinline__ bool
fix_any(const xa_dec_args &a, uint32_t fmt, uint32_t q, uint2 s, uint2 &ex)
{
	const int64_t bb = (int64_t)q * a.C;
	switch (fmt) {
	case 8 | 2 << 8:
		return fix_chunk<8, 2>(a, q, s, ex, bb);
	case 6 | 2 << 8:
		return fix_chunk<6, 2>(a, q, s, ex, bb);
	case 4 | 2 << 8:
		return fix_chunk<4, 2>(a, q, s, ex, bb);
	case 8 | 1 << 8:
		return fix_chunk<8, 1>(a, q, s, ex, bb);
	case 6 | 1 << 8:
		return fix_chunk<6, 1>(a, q, s, ex, bb);
	default:
		return fix_chunk<4, 1>(a, q, s, ex, bb);
	}
}

/* global chunk Q is no boundary of its stream (the stream's chunk 0, or a
 * padding slot of its last wave) */
__device__ __forceinline__ bool
batch_no_boundary(const xa_batch_args &b, uint32_t Q)
{
	const xa_batch_stream &d = b.streams[b.wstream[Q / 64]];
	const uint32_t q = Q - d.cbase;
	return q == 0 || q >= d.nchunks;
}

/*
 * Sequential tail of a batch (thread 0): drain the re-check queue in global
 * chunk order.  Global chunk indices never cross streams (a stream's chunk
 * 0 is never queued); entries that are no boundary (stale ones) are
 * skipped.
 */
__device__ __forceinline__ void
drain_batch(const xa_batch_args &b)
{
	const uint32_t nc = 64u * b.nwaves, nq = min(b.ctl[XA_CTL_NQ], 2u * nc);
	uint32_t n = 0;
	for (uint32_t i = 0; i < nq; i++) {
		const uint32_t Q = b.queue[i];
		if (Q >= 1u && Q < nc && !batch_no_boundary(b, Q))
			heap_push(b.queue, n, Q);
	}
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
		if (!met) {
			b.e[Q] = ex;
			if (q + 1 < a.nchunks)
				heap_push(b.queue, n, Q + 1);
		}
	}
}

/*
 * K2 over a batch: one workgroup drains what the batch K1 queued, in global
 * chunk order, repairing in each chunk's stream format, then publishes every
 * stream's status.
 */
__global__ __launch_bounds__(XA_TAIL_THREADS) void
xa_decode_tail_batch(xa_batch_args b)
{
	if (b.ctl[XA_CTL_OVF] != 0u)
		rebuild_queue(b.e, b.g, b.queue, &b.ctl[XA_CTL_NQ], 1u,
		    64u * b.nwaves, [&](uint32_t Q) {
			    return batch_no_boundary(b, Q);
		    });
	else
		filter_queue(b.queue, &b.ctl[XA_CTL_NQ], 2u * 64u * b.nwaves,
		    [&](uint32_t Q) {
			    return Q >= 1u && Q < 64u * b.nwaves &&
				!batch_no_boundary(b, Q) && differs(b.e, b.g, Q);
		    });
	if (threadIdx.x == 0)
		drain_batch(b);
	__syncthreads();
	/* every stream's status: up to XA_PUB streams per thread, each loaded
	 * in full before any is written, so the dependent loads (descriptor,
	 * then the last chunk's exit state) overlap across streams */
	constexpr int XA_PUB = 4;
	for (uint32_t s0 = 0; s0 < b.nstreams; s0 += XA_TAIL_THREADS * XA_PUB) {
		uint32_t err[XA_PUB], fix[XA_PUB], tail[XA_PUB], nch[XA_PUB], cc[XA_PUB];
		uint2 fin[XA_PUB];
#pragma unroll
		for (int j = 0; j < XA_PUB; j++) {
			const uint32_t s = min(s0 + threadIdx.x + XA_TAIL_THREADS * j,
			    b.nstreams - 1);
			const xa_batch_stream &dd = b.streams[s];
			const uint32_t *sc = b.sctl + s * XA_SCTL_WORDS;
			nch[j] = dd.nchunks;
			cc[j] = dd.C;
			fin[j] = b.e[dd.cbase + dd.nchunks - 1];
			err[j] = sc[XA_SCTL_ERR];
			fix[j] = sc[XA_SCTL_FIXED];
			tail[j] = sc[XA_SCTL_TAIL];
		}
#pragma unroll
		for (int j = 0; j < XA_PUB; j++) {
			const uint32_t s = s0 + threadIdx.x + XA_TAIL_THREADS * j;
			if (s >= b.nstreams)
				continue;
			uint32_t *sc = b.sctl + s * XA_SCTL_WORDS;
			uint32_t *st = b.status + s * XA_ST_WORDS;
			st[XA_ST_ERR] = err[j];
			st[XA_ST_STATE_L] = fin[j].x;
			st[XA_ST_STATE_R] = fin[j].y;
			st[XA_ST_FIXED] = fix[j];
			st[XA_ST_TAIL] = tail[j];
			st[XA_ST_CHUNKS] = nch[j];
			st[XA_ST_C] = cc[j];
			st[XA_ST_W] = b.W;
			sc[XA_SCTL_ERR] = 0xffffffffu;
			sc[XA_SCTL_FIXED] = 0;
			sc[XA_SCTL_TAIL] = 0;
		}
	}
	if (threadIdx.x == 0) {
		b.ctl[XA_CTL_NQ] = 0;
		b.ctl[XA_CTL_OVF] = 0;
	}
}

hipError_t
xa_decode_batch_launch(const xa_batch_args &b0, hipStream_t st, hipEvent_t ev0,
    hipEvent_t ev1)
{
	xa_batch_args b = b0;
	b.tag = next_tag();
	const unsigned grid = (b.nwaves + XA_SPEC_WPB - 1) / XA_SPEC_WPB;
	if (ev0 != NULL)
		(void)hipEventRecord(ev0, st);
	hipLaunchKernelGGL(xa_decode_spec_batch, dim3(grid), dim3(XA_SPEC_CPW), 0,
	    st, b);
	if (ev1 != NULL)
		(void)hipEventRecord(ev1, st);
	hipLaunchKernelGGL(xa_decode_tail_batch, dim3(1), dim3(XA_TAIL_THREADS),
	    0, st, b);
	return hipGetLastError();
}
