/*
 * xa_encode.hip -- gfx950 XA encode.
 *
 * Replaces bjxa_encode (reference src/libbjxa.c:759-819) ->
 * bjxa_encode_inflated (:665-691) -> bjxa_deflate_{4,6,8}bits (:349-391).
 * The reference encoder writes profile 0 (gain 0, range 0: :679) and keeps
 * the top `bits` bits of every sample, zero-padding the last block.  There
 * is no state and no dependency between blocks, so this is pure streaming:
 * one lane packs one 4-block group (256 B of PCM -> 4*(bits*4+1) B of XA,
 * a whole number of dwords).
 */
#include "xa_common.h"
#include "xa_decode.h"

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(16)));

/* top `BITS` bits of int16 sample k (0..127) of the group, right-aligned */
template <int BITS>
__device__ __forceinline__ uint32_t
enc_code(const uint32_t *pcm, const int k)
{
	return (pcm[k >> 1] >> (16 * (k & 1) + 16 - BITS)) & ((1u << BITS) - 1u);
}

/* byte p (0 .. 4*BSZ-1) of the packed group */
template <int BITS, int CH>
__device__ __forceinline__ uint32_t
enc_byte(const uint32_t *pcm, const int p)
{
	constexpr int BSZ = BITS * 4 + 1;
	const int cb = p / BSZ, j = p % BSZ - 1;
	if (j < 0)
		return 0u;		/* profile byte (src/libbjxa.c:679) */
	const int u = cb / CH, c = cb % CH;
	/* sample of frame n of this channel block */
#define SMP(n) ((u * XA_FRAMES + (n)) * CH + c)
	if (BITS == 8)
		return enc_code<8>(pcm, SMP(j));
	if (BITS == 4)
		return (enc_code<4>(pcm, SMP(2 * j)) << 4) |
		    enc_code<4>(pcm, SMP(2 * j + 1));
	/* 6-bit: byte j of the big-endian 24-bit groups of four codes */
	const int gi = j / 3, r = j % 3;
	const uint32_t g24 = (enc_code<6>(pcm, SMP(4 * gi)) << 18) |
	    (enc_code<6>(pcm, SMP(4 * gi + 1)) << 12) |
	    (enc_code<6>(pcm, SMP(4 * gi + 2)) << 6) |
	    enc_code<6>(pcm, SMP(4 * gi + 3));
	return (g24 >> (16 - 8 * r)) & 0xffu;
#undef SMP
}

template <int BITS, int CH>
__global__ __launch_bounds__(256) void
xa_encode_groups(xa_enc_args a)
{
	constexpr int BSZ = BITS * 4 + 1, G = 4 / CH, GDW = BSZ;
	const uint64_t grp = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	const uint64_t ngroups = ((uint64_t)a.eblocks + G - 1) / G;
	if (grp >= ngroups)
		return;
	const uint64_t f0 = grp * G * XA_FRAMES;	/* first frame */
	uint32_t pcm[64];
	const uint32_t *sp = (const uint32_t *)(a.src + f0 * CH * 2);
	if (f0 + G * XA_FRAMES <= a.frames) {
#pragma unroll
		for (int i = 0; i < 16; i++) {
			u32x4a v = ((const u32x4a *)sp)[i];
			pcm[4 * i] = v.x;
			pcm[4 * i + 1] = v.y;
			pcm[4 * i + 2] = v.z;
			pcm[4 * i + 3] = v.w;
		}
	} else {
		/* last group: frames past the end encode as 0 (:686-690) */
		const uint64_t nsmp = (a.frames - f0) * CH;
		const uint16_t *hp = (const uint16_t *)sp;
#pragma unroll
		for (int i = 0; i < 64; i++) {
			uint32_t lo = (uint64_t)(2 * i) < nsmp ? hp[2 * i] : 0u;
			uint32_t hi = (uint64_t)(2 * i + 1) < nsmp ? hp[2 * i + 1] : 0u;
			pcm[i] = lo | (hi << 16);
		}
	}
	uint32_t out[GDW];
#pragma unroll
	for (int d = 0; d < GDW; d++) {
		out[d] = enc_byte<BITS, CH>(pcm, 4 * d) |
		    (enc_byte<BITS, CH>(pcm, 4 * d + 1) << 8) |
		    (enc_byte<BITS, CH>(pcm, 4 * d + 2) << 16) |
		    (enc_byte<BITS, CH>(pcm, 4 * d + 3) << 24);
	}
	/* the group may run past the last eblock: write only real blocks */
	uint32_t *dp = (uint32_t *)(a.dst + grp * 4 * BSZ);
	const uint64_t blocks_here = ((uint64_t)a.eblocks - grp * G) < (uint64_t)G ?
	    ((uint64_t)a.eblocks - grp * G) : (uint64_t)G;
	if (blocks_here == (uint64_t)G) {
#pragma unroll
		for (int d = 0; d < GDW; d++)
			dp[d] = out[d];
	} else {
		const int nbytes = (int)blocks_here * CH * BSZ;
		uint8_t *bp = (uint8_t *)dp;
#pragma unroll
		for (int d = 0; d < GDW; d++)
#pragma unroll
			for (int k = 0; k < 4; k++)
				if (4 * d + k < nbytes)
					bp[4 * d + k] = (uint8_t)(out[d] >> (8 * k));
	}
}

hipError_t
xa_encode_launch(const xa_enc_args &a, unsigned bits, unsigned ch,
    hipStream_t st)
{
	const uint64_t G = 4 / ch;
	const uint64_t ngroups = ((uint64_t)a.eblocks + G - 1) / G;
	const unsigned grid = (unsigned)((ngroups + 255) / 256);
	if (grid == 0)
		return hipSuccess;
#define L(B, C) hipLaunchKernelGGL((xa_encode_groups<B, C>), dim3(grid), \
    dim3(256), 0, st, a)
	if (ch == 1) {
		if (bits == 8) L(8, 1); else if (bits == 6) L(6, 1); else L(4, 1);
	} else {
		if (bits == 8) L(8, 2); else if (bits == 6) L(6, 2); else L(4, 2);
	}
#undef L
	return hipGetLastError();
}
