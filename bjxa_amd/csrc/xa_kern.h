/*
 * xa_kern.h -- device building blocks of the decode kernels
 * (xa_decode.hip: K1, K2 and their batch forms).  Internal.
 */
#ifndef BJXA_XA_KERN_H
#define BJXA_XA_KERN_H

#include <type_traits>

#include "xa_common.h"
#include "xa_decode.h"

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
	static constexpr int G2 = XA_CHUNK_Q(CH);	/* chunk granularity */
	static constexpr int GDW = BSZ;			/* dwords per group */
	static constexpr int OB = 64 * CH;		/* PCM bytes per eblock */
};

/*
 * Decode the channel blocks of one eblock whose first byte is byte O of w,
 * advancing the lane's state.  With STORE the output goes to `line` in
 * 16-B pieces, numbered from QB (the eblock's first piece within the
 * group); after every LB bytes `flush(h)` runs (h = LB-byte line index
 * within the group), and with RESTART the next line is written at `line`
 * again (LDS staging), otherwise output continues at line + LB (direct
 * stores).  A line may span eblocks (mono: 64 B per block).  Returns a bit
 * per channel whose gain nibble is >= 5.
 */
template <int BITS, int CH, bool STORE, bool RESTART, int LB, int QB = 0,
    typename F>
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
	/* f32 state for the block (xa_common.h): stereo runs both chains in
	 * one packed instruction stream (xa_step_lr), mono one chain
	 * (xa_step_f); the int state converts in and out once per eblock.
	 * shp: the range of each half of a packed code pair (mono: both
	 * halves are the block's one range) */
	xa_f2 f0 = {(float)p0[0], (float)p0[CH - 1]};
	xa_f2 f1 = {(float)p1[0], (float)p1[CH - 1]};
	const xa_f2 fk0 = xa_f2{(float)k0[0], (float)k0[CH - 1]} * (1.0f / 256.0f);
	const xa_f2 fk1 = xa_f2{(float)k1[0], (float)k1[CH - 1]} * (1.0f / 256.0f);
	const uint32_t shp = (sh[0] - 16u) | ((sh[CH - 1] - 16u) << 16);
	float m0 = f0.x, m1 = f1.x;	/* mono state */
	/* 16-B piece q holds 4 stereo frames or 8 mono samples */
#pragma unroll
	for (int q = 0; q < 4 * CH; q++) {
		uint32_t fr[4];
#pragma unroll
		for (int j = 0; j < 4; j++) {
			if (CH == 2) {
				const int n = 4 * q + j;
				uint32_t tp;
				if (BITS == 8) {
					/* code n of L -> bits 8..15, of R -> 24..31 */
					const int bl = O + 1 + n, br = O + BSZ + 1 + n;
					tp = __builtin_amdgcn_perm(w[br >> 2], w[bl >> 2],
					    0x000c000cu | (uint32_t)(bl & 3) << 8 |
					    (uint32_t)(4 + (br & 3)) << 24);
				} else {
					tp = __builtin_amdgcn_perm(
					    (uint32_t)code_at<BITS>(w, O + BSZ, n),
					    (uint32_t)code_at<BITS>(w, O, n), 0x07060302u);
				}
				fr[j] = xa_step_lr(xa_pk_ashr(tp, shp), fk0, fk1, f0, f1);
			} else {
				/* codes n, n+1 into the halves, one packed shift */
				const int n = 8 * q + 2 * j;
				uint32_t tp;
				if (BITS == 8) {
					const int b = O + 1 + n;
					tp = __builtin_amdgcn_perm(w[(b + 1) >> 2],
					    w[b >> 2], 0x000c000cu |
					    (uint32_t)(b & 3) << 8 |
					    (uint32_t)(((b + 1) >> 2) == (b >> 2) ?
					    (b + 1) & 3 : 4 + ((b + 1) & 3)) << 24);
				} else {
					tp = __builtin_amdgcn_perm(
					    (uint32_t)code_at<BITS>(w, O, n + 1),
					    (uint32_t)code_at<BITS>(w, O, n), 0x07060302u);
				}
				const uint32_t t = xa_pk_ashr(tp, shp);
				int32_t sa = xa_step_f<false>(t, fk0.x, fk1.x, m0, m1);
				int32_t sb = xa_step_f<true>(t, fk0.x, fk1.x, m0, m1);
				fr[j] = __builtin_amdgcn_perm((uint32_t)sb,
				    (uint32_t)sa, 0x05040100u);
			}
		}
		if (STORE) {
			u32x4a v = { fr[0], fr[1], fr[2], fr[3] };
			constexpr int QL = LB / 16;	/* pieces per line */
			const int qq = QB + q;
			/* (RESTART: the stage's piece order, pieces 4-7 of a
			 * line 64 B further -- xa_decode.hip ost_piece) */
			static_assert(!STORE || !RESTART || QL == 8, "stage piece order");
			*(u32x4a *)(line + 16 * (RESTART ? (qq % QL) + (qq % QL & 4) : qq)) = v;
			if (qq % QL == QL - 1)
				flush(qq / QL);
		}
		/* keep the unpack of later codes from being hoisted here: it
		 * would only raise register pressure */
		__builtin_amdgcn_sched_barrier(0);
	}
	if (CH == 1) {
		p0[0] = (int32_t)m0;
		p1[0] = (int32_t)m1;
	}
	if (CH == 2) {
		p0[0] = (int32_t)f0.x;
		p0[CH - 1] = (int32_t)f0.y;
		p1[0] = (int32_t)f1.x;
		p1[CH - 1] = (int32_t)f1.y;
	}
	return bad;
}

/* one LDS-DMA instruction of PS bytes per lane (the builtin wants a
 * literal size) */
template <int PS> __device__ __forceinline__ void dma(const void *, uint8_t *);
template <> __device__ __forceinline__ void
dma<4>(const void *g, uint8_t *l)
{
	__builtin_amdgcn_global_load_lds(g, LDS_PTR(l), 4, 0, XA_DMA_AUX);
}
template <> __device__ __forceinline__ void
dma<16>(const void *g, uint8_t *l)
{
	__builtin_amdgcn_global_load_lds(g, LDS_PTR(l), 16, 0, XA_DMA_AUX);
}

#endif
