/*
 * xa_region.hip -- gfx950 region decode (K1r): the automatic decode kernel
 * of bjxa_hip_decode_async for one stream.  See the comment below and
 * DESIGN.md §3; K2 (xa_decode.hip) verifies the region boundaries.
 */
#include "xa_kern.h"

/* ------------------------------------------------------------------ */
/* K1r: region decode -- contiguous input per wave, in-wave verification */

/*
 * The lane-strided K1 above reads, at every super-step, 64 separate 264-B
 * runs per wave (one per lane's chunk), and the counters show what that
 * costs: every run straddles 128-B lines and the shared line is fetched
 * again (L2->fabric reads 1.44x the stream at warm-up 0, 1.73x with the
 * warm-up re-read; tools/rdreq_calib.hip).
 *
 * K1r turns the access inside out.  A wave owns a *region* of 64 short
 * chunks of C eblocks (C * EBSZ = 528 B for 8-bit stereo), i.e. one
 * contiguous run of the stream; the W eblocks before the region come with
 * it.  The whole region lands in LDS by LDS-DMA in 1-KiB contiguous
 * instructions.  Lane m's warm-up is lane m-1's chunk, read straight from
 * the image: it costs decode work (W = C for stereo: twice the predictor
 * steps) but no extra HBM read, and every input line is fetched once.  Then
 * each lane copies its own chunk (C * EBSZ bytes, 33 dwordx4 for 8-bit
 * stereo) into registers and the next region's DMA is issued, so it lands
 * while this region's chunks decode.  One wave per SIMD (4 per CU, one
 * workgroup per CU: ~154 KiB of LDS) leaves each lane the whole register
 * file (the compiler keeps the chunk partly in AGPRs), and a persistent
 * grid keeps the DMA of region r+1 in flight behind the decode of r.
 *
 * Verification moves into the wave: lane m's entry state (after its warm-up
 * over lane m-1's chunk from (0,0)) must equal lane m-1's exit state; a
 * lane where it does not re-decodes its chunk from its neighbour's exit
 * (the input is still in its VGPRs) until its block-end states meet the
 * stored trajectory, re-storing the blocks it changed, and a changed exit
 * makes its successor check again.  What is left for K2 is one boundary per
 * region (lane 0's warm-up entry against the previous region's exit), so K2
 * runs unchanged with regions as its chunks (64 * C eblocks).
 */
template <int BITS, int CH> struct rgeo {
	typedef geo<BITS, CH> g;
	static constexpr int EBSZ = g::EBSZ, OB = g::OB;
	static constexpr int C = XA_REGION_C(CH);	/* lane chunk, eblocks */
	static constexpr int W = XA_REGION_W;		/* warm-up, eblocks */
	static constexpr int LANEB = (C + W) * EBSZ;	/* input bytes per lane */
	static constexpr int OWN = W * EBSZ;		/* the chunk's byte in a lane's run */
	static constexpr int RD = C * EBSZ / 4;		/* the chunk's dwords (VGPRs) */
	static constexpr int NPL = (LANEB + 15) / 16;	/* 16-B pieces per lane run */
	static constexpr int IMG = (64 * C + W) * EBSZ;	/* region image, bytes */
	static constexpr int IMGP = (IMG + 15) / 16;	/* its 16-B pieces */
	static constexpr int NI = (IMGP + 63) / 64;	/* DMA instructions */
	static constexpr int LASTL = IMGP - 64 * (NI - 1);	/* lanes of the last */
	static constexpr int IMGA = NI * 1024;		/* LDS image bytes */
	static constexpr int U = 128 / OB;		/* eblocks per 128-B line */
	static constexpr int NU = C / U;		/* lines per lane per region */
	static constexpr int LINE = 144;		/* staged line stride */
	static constexpr int REGION = IMGA + 32 * LINE;	/* LDS per wave */
	static_assert((C * EBSZ) % 16 == 0, "lane runs start 16-B aligned");
	static_assert(OWN % 4 == 0, "the chunk starts on a dword");
	static_assert(63 * C * EBSZ + NPL * 16 <= IMGA, "lane copy inside the image");
	static_assert(C * OB == 1024, "a lane's chunk is 1 KiB of PCM");
	static_assert(4 * REGION <= 160 * 1024, "one workgroup per CU");
};

#define XA_REGION_WAVES 4	/* waves per workgroup: one per SIMD */

/*
 * N dwords from LDS at p, whose address is A mod 16 (compile time): dword
 * reads up to the first 16-B boundary, then ds_read_b128, then the tail
 */
template <int N, int A>
__device__ __forceinline__ void
lds_read_dw(const uint8_t *p, uint32_t *out)
{
	static_assert(A % 4 == 0, "dword aligned");
	constexpr int H = ((16 - A) % 16) / 4 < N ? ((16 - A) % 16) / 4 : N;
	constexpr int B = (N - H) / 4;
#pragma unroll
	for (int i = 0; i < H; i++)
		out[i] = ((const uint32_t *)p)[i];
#pragma unroll
	for (int i = 0; i < B; i++) {
		const u32x4a v = *(const u32x4a *)(p + 4 * H + 16 * i);
		out[H + 4 * i] = v.x;
		out[H + 4 * i + 1] = v.y;
		out[H + 4 * i + 2] = v.z;
		out[H + 4 * i + 3] = v.w;
	}
#pragma unroll
	for (int i = H + 4 * B; i < N; i++)
		out[i] = ((const uint32_t *)p)[i];
}

/* land region r's image (eblocks rs - W .. rs + 64C) in LDS */
template <int BITS, int CH>
__device__ __forceinline__ void
region_stage(const xa_dec_args &a, uint8_t *img, int lane, int64_t rs)
{
	typedef rgeo<BITS, CH> R;
	const int64_t b0 = (rs - R::W) * R::EBSZ;	/* stream byte of image byte 0 */
	const int64_t nbytes = (int64_t)a.eblocks * R::EBSZ;
	if (b0 >= 0 && b0 + R::IMGP * 16 <= nbytes) {
		const uint8_t *base = a.src + b0 + lane * 16;
#pragma unroll
		for (int i = 0; i < R::NI; i++)
			if (i < R::NI - 1 || lane < R::LASTL)
				dma<16>(base + i * 1024, img + i * 1024);
		return;
	}
	/* the first and last regions: dword pieces, each clamped into the
	 * stream (the dword holding the last byte is read whole, as in
	 * stage_half); bytes outside the stream are never decoded into PCM */
	int64_t bb = b0, lim = nbytes;
	const uint8_t *src = a.src;
	asm volatile("" : "+v"(bb), "+v"(lim), "+v"(src));
	const int64_t last = (lim - 1) & ~(int64_t)3;
#pragma nounroll
	for (int i = 0; i < (R::IMGP * 4 + 63) / 64; i++) {
		const int k = i * 64 + lane;
		if (k >= R::IMGP * 4)
			continue;
		int64_t byte = bb + 4 * (int64_t)k;
		byte = byte < 0 ? 0 : (byte > last ? last : byte);
		dma<4>(src + byte, img + i * 256);
	}
}

/*
 * Store line u (128 B: eblock u*U .. u*U+U-1 of each lane's chunk) of the
 * wave's 64 chunks, staged half a wave at a time so that every store
 * instruction covers 8 whole lines.  `v` holds the lane's line (8 pieces);
 * `own` says whether the lane's line is to be written (repairs); `fast`
 * (wave-uniform): the region's PCM is whole and every line is written.
 */
template <int BITS, int CH>
__device__ __forceinline__ void
region_store(const xa_dec_args &a, uint8_t *stg, int lane, uint32_t q0,
    int u, const uint32_t *v, bool own, bool fast)
{
	typedef rgeo<BITS, CH> R;
	constexpr int LINE = R::LINE;
	/* the lane's piece of the lines it stores: line 8i + lane/8 of the
	 * half, piece lane % 8 */
	const int pc = lane & 7, lj = lane >> 3;
#pragma unroll
	for (int h = 0; h < 2; h++) {
		if ((lane >> 5) == h) {
			uint8_t *d = stg + (lane & 31) * LINE;
#pragma unroll
			for (int p = 0; p < 8; p++)
				*(u32x4a *)(d + 16 * p) = u32x4a{v[4 * p], v[4 * p + 1],
				    v[4 * p + 2], v[4 * p + 3]};
			if (!fast)
				*(uint32_t *)(d + 128) = own ? 1u : 0u;
		}
		wave_lds_sync();
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint8_t *s = stg + (8 * i + lj) * LINE;
			const u32x4a w = *(const u32x4a *)(s + 16 * pc);
			const uint32_t qq = q0 + 32u * h + 8u * i + (uint32_t)lj;
			const uint64_t off = (uint64_t)qq * 1024u + (uint64_t)u * 128u +
			    16u * pc;
			if (fast) {
				__builtin_nontemporal_store(w, (u32x4a *)(a.dst + off));
			} else {
				const bool wr = *(const uint32_t *)(s + 128) != 0u;
				if (!wr || qq >= a.nchunks)
					continue;
				if (off + 16u <= a.pcm_bytes) {
					__builtin_nontemporal_store(w, (u32x4a *)(a.dst + off));
				} else if (off < a.pcm_bytes) {
					const uint32_t ww[4] = { w.x, w.y, w.z, w.w };
#pragma unroll
					for (int k = 0; k < 8; k++)
						if (off + 2u * k < a.pcm_bytes)
							*(uint16_t *)(a.dst + off + 2u * k) =
							    (uint16_t)(ww[k >> 1] >> (16 * (k & 1)));
				}
			}
		}
		/* the staged lines have been read back before the next half
		 * overwrites them */
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		wave_lds_sync();
	}
}

/* pack / unpack a lane's per-channel state words */
template <int CH>
__device__ __forceinline__ void
region_pack(const int32_t *p0, const int32_t *p1, uint32_t *s)
{
#pragma unroll
	for (int c = 0; c < CH; c++)
		s[c] = xa_pack_state(p0[c], p1[c]);
}

/*
 * One region r of the wave: decode from the lane's VGPR copy `rg` (warm-up
 * eblocks at byte 0, the chunk at byte W * EBSZ), store, verify in-wave and
 * repair.  Writes g[r] (lane 0's entry state) and e[r] (the exit state of
 * the region's last chunk).
 */
template <int BITS, int CH, typename F>
__device__ __forceinline__ void
region_decode(const xa_dec_args &a, const uint8_t *img, uint8_t *stg, int lane,
    uint32_t r, bool fast, F &&next_dma)
{
	typedef rgeo<BITS, CH> R;
	constexpr int C = R::C, W = R::W, EBSZ = R::EBSZ, U = R::U, NU = R::NU;
	const uint32_t q0 = r * 64u, q = q0 + (uint32_t)lane;
	const int64_t eblocks = a.eblocks;
	const int64_t b0 = (int64_t)q * C;
	const uint8_t *run = img + lane * (C * EBSZ);	/* 16-B aligned */
	auto none = [](int) {};

	int32_t p0[CH], p1[CH];
#pragma unroll
	for (int c = 0; c < CH; c++)
		p0[c] = p1[c] = 0;
	/* warm-up over the W eblocks before the chunk (lane m-1's chunk),
	 * from (0,0), read straight from the image; chunk 0 takes the
	 * caller's state instead */
	auto warm = [&](auto kc) {
		constexpr int k = decltype(kc)::value;
		constexpr int D0 = k * EBSZ / 4, DN = ((k + 1) * EBSZ + 3) / 4 - D0;
		uint32_t wk[DN];
		lds_read_dw<DN, (4 * D0) % 16>(run + 4 * D0, wk);
		(void)decode_eblock<BITS, CH, false, true, 64>(wk, k * EBSZ - 4 * D0,
		    p0, p1, nullptr, none);
	};
	sfor<0, W>::run(warm);
	/* the chunk itself into VGPRs; then the image is free for the next
	 * region's DMA, which lands while this region decodes */
	uint32_t rg[R::RD];
	lds_read_dw<R::RD, R::OWN % 16>(run + R::OWN, rg);
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	next_dma();
	asm volatile("" ::: "memory");
	if (q == 0) {
#pragma unroll
		for (int c = 0; c < CH; c++)
			xa_unpack_state(a.init[c], p0[c], p1[c]);
	}
	uint32_t ent[CH];
	region_pack<CH>(p0, p1, ent);
	const uint32_t gst0 = ent[0], gst1 = ent[CH - 1];

	/* the chunk: block-end states kept for the in-wave repair */
	uint32_t bend[C][CH];
	auto unit = [&](auto uc) {
		constexpr int u = decltype(uc)::value;
		uint32_t v[32];
		auto blk = [&](auto jc) {
			constexpr int j = decltype(jc)::value, k = u * U + j;
			const int64_t b = b0 + k;
			int32_t q0s[CH], q1s[CH];
#pragma unroll
			for (int c = 0; c < CH; c++) {
				q0s[c] = p0[c];
				q1s[c] = p1[c];
			}
			const uint32_t bad = decode_eblock<BITS, CH, true, false, 128,
			    j * 4 * CH>(rg, k * EBSZ, p0, p1, (uint8_t *)v, none);
			const bool act = b < eblocks;
			if (act && bad) {
				const uint32_t cb = (uint32_t)b * CH + ((bad & 1u) ? 0u : 1u);
				atomicMin(&a.ctl[XA_CTL_ERR], cb);
			}
#pragma unroll
			for (int c = 0; c < CH; c++) {
				p0[c] = act ? p0[c] : q0s[c];
				p1[c] = act ? p1[c] : q1s[c];
			}
			region_pack<CH>(p0, p1, bend[k]);
		};
		sfor<0, U>::run(blk);
		region_store<BITS, CH>(a, stg, lane, q0, u, v, true, fast);
	};
	sfor<0, NU>::run(unit);

	/* in-wave verification: lane m's entry against lane m-1's exit */
	const bool has = b0 < eblocks;
	uint32_t nrep = 0;
#ifdef XA_DBG_NOREP
	/* diagnostic builds only: no in-wave repair (wrong output on
	 * mismatching chunks) */
	for (; false;) {
#else
	for (;;) {
#endif
		bool need = false;
		uint32_t prev[CH];
#pragma unroll
		for (int c = 0; c < CH; c++) {
			prev[c] = (uint32_t)__shfl_up((int)bend[C - 1][c], 1);
			need = need || prev[c] != ent[c];
		}
		need = need && lane > 0 && has;
		const uint64_t nb = __ballot(need);
		if (nb == 0)
			break;
		nrep += (uint32_t)__builtin_popcountll(nb);
#pragma unroll
		for (int c = 0; c < CH; c++) {
			ent[c] = need ? prev[c] : ent[c];
			xa_unpack_state(ent[c], p0[c], p1[c]);
		}
		/* re-decode from the true entry until a line-end state meets the
		 * stored trajectory; lines the lane changed are stored again */
		bool active = need;
		auto rep = [&](auto uc) {
			constexpr int u = decltype(uc)::value;
			if (__ballot(active) == 0)
				return;
			uint32_t v[32];
			bool met = false;
			auto blk = [&](auto jc) {
				constexpr int j = decltype(jc)::value, k = u * U + j;
				const int64_t b = b0 + k;
				int32_t q0s[CH], q1s[CH];
#pragma unroll
				for (int c = 0; c < CH; c++) {
					q0s[c] = p0[c];
					q1s[c] = p1[c];
				}
				/* fresh copies of the block's input words: without them
				 * the compiler keeps the main pass's unpacked codes of
				 * every block alive for this rare path (and spills) */
				constexpr int D0 = (k * EBSZ) / 4;
				constexpr int DN = ((k + 1) * EBSZ + 3) / 4 - D0;
				uint32_t wk[DN];
#pragma unroll
				for (int i = 0; i < DN; i++) {
					wk[i] = rg[D0 + i];
					asm volatile("" : "+v"(wk[i]));
				}
				(void)decode_eblock<BITS, CH, true, false, 128, j * 4 * CH>(wk,
				    k * EBSZ - 4 * D0, p0, p1, (uint8_t *)v, none);
				const bool act = b < eblocks;
#pragma unroll
				for (int c = 0; c < CH; c++) {
					p0[c] = act ? p0[c] : q0s[c];
					p1[c] = act ? p1[c] : q1s[c];
				}
				uint32_t nsw[CH];
				region_pack<CH>(p0, p1, nsw);
				bool same = act;
#pragma unroll
				for (int c = 0; c < CH; c++) {
					same = same && nsw[c] == bend[k][c];
					bend[k][c] = active ? nsw[c] : bend[k][c];
				}
				/* a meeting counts at the line's last block: the line is
				 * stored whole, and after a meeting the decode reproduces
				 * the stored PCM */
				if (j == U - 1)
					met = same;
			};
			sfor<0, U>::run(blk);
			region_store<BITS, CH>(a, stg, lane, q0, u, v, active, false);
			active = active && !met;
		};
		sfor<0, NU>::run(rep);
	}
	if (lane == 0 && nrep)
		atomicAdd(&a.ctl[XA_CTL_FIXED], nrep);
	/* K2's view: the region's entry (lane 0) and exit (its last chunk) */
	const uint32_t lastq = min(q0 + 63u, a.nchunks - 1u) - q0;
	const uint32_t ex0 = __shfl((int)bend[C - 1][0], (int)lastq);
	const uint32_t ex1 = __shfl((int)bend[C - 1][CH - 1], (int)lastq);
	if (lane == 0) {
		a.g[r] = make_uint2(gst0, CH == 2 ? gst1 : 0u);
		a.e[r] = make_uint2(ex0, CH == 2 ? ex1 : 0u);
	}
}

/* K1r: persistent; wave w takes regions w, w + nwaves, ... */
template <int BITS, int CH>
__global__ __launch_bounds__(64 * XA_REGION_WAVES, 1) void
xa_decode_region(xa_dec_args a, uint32_t nreg)
{
	typedef rgeo<BITS, CH> R;
	__shared__ __attribute__((aligned(16))) uint8_t
	    lds[XA_REGION_WAVES * R::REGION];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *img = lds + wv * R::REGION, *stg = img + R::IMGA;
	const uint32_t nw = gridDim.x * XA_REGION_WAVES;
	uint32_t r = blockIdx.x * XA_REGION_WAVES + (uint32_t)wv;
	if (r >= nreg)
		return;
	const uint64_t full_blocks = a.pcm_bytes / R::OB;
	region_stage<BITS, CH>(a, img, lane, (int64_t)r * 64 * R::C);
	bool fast_prev = false;	/* the previous region stored on the fast path */
	for (; r < nreg; r += nw) {
		/* this region's image has landed: leave the previous region's
		 * stores (at least 64, all younger than the DMA) in flight */
		if (fast_prev)
			asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
		else
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		/* fast: every chunk of the region is whole and inside the PCM */
		const bool fast = (uint64_t)(r + 1) * 64u * R::C <= full_blocks;
		const uint32_t rn = r + nw;
		region_decode<BITS, CH>(a, img, stg, lane, r, fast, [&] {
			if (rn < nreg)
				region_stage<BITS, CH>(a, img, lane, (int64_t)rn * 64 * R::C);
		});
		fast_prev = fast;
	}
}

template <int BITS, int CH>
static hipError_t
launch_region(const xa_dec_args &a, unsigned ncu, hipStream_t st, hipEvent_t ev0,
    hipEvent_t ev1)
{
	typedef rgeo<BITS, CH> R;
	const uint32_t nreg = (a.nchunks + 63u) / 64u;
	uint32_t waves = ncu * XA_REGION_WAVES;
	if (waves > nreg)
		waves = nreg;
	const unsigned grid = (waves + XA_REGION_WAVES - 1) / XA_REGION_WAVES;
	if (ev0 != NULL)
		(void)hipEventRecord(ev0, st);
	hipLaunchKernelGGL((xa_decode_region<BITS, CH>), dim3(grid),
	    dim3(64 * XA_REGION_WAVES), 0, st, a, nreg);
	if (ev1 != NULL)
		(void)hipEventRecord(ev1, st);
#if !defined(XA_DBG_STEP) && !defined(XA_DBG_NOSTORE) && !defined(XA_DBG_CONTIG)
	/* K2 over regions: chunk = region (64 * C eblocks) */
	xa_dec_args k2 = a;
	k2.C = 64u * R::C;
	k2.nchunks = nreg;
	k2.nlong = 0;
	k2.rep_C = R::C;
	k2.rep_chunks = a.nchunks;
	const hipError_t e2 = xa_decode_fix_launch(k2, BITS, CH, st);
	if (e2 != hipSuccess)
		return e2;
#endif
	return hipGetLastError();
}

hipError_t
xa_decode_region_launch(const xa_dec_args &a, unsigned bits, unsigned ch,
    unsigned ncu, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1)
{
#ifdef XA_REGION_ONLY82
	/* quick builds for kernel experiments (tools/kres.py): 8-bit stereo */
	(void)bits;
	(void)ch;
	return launch_region<8, 2>(a, ncu, st, ev0, ev1);
#else
	if (ch == 1) {
		if (bits == 8)
			return launch_region<8, 1>(a, ncu, st, ev0, ev1);
		if (bits == 6)
			return launch_region<6, 1>(a, ncu, st, ev0, ev1);
		return launch_region<4, 1>(a, ncu, st, ev0, ev1);
	}
	if (bits == 8)
		return launch_region<8, 2>(a, ncu, st, ev0, ev1);
	if (bits == 6)
		return launch_region<6, 2>(a, ncu, st, ev0, ev1);
	return launch_region<4, 2>(a, ncu, st, ev0, ev1);
#endif
}
