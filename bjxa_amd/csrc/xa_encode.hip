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

#define XA_ENC_WPB 4		/* waves per workgroup */
#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))

__device__ __forceinline__ void
wave_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int BITS, int CH>
__global__ __launch_bounds__(64 * XA_ENC_WPB) void
xa_encode_waves(xa_enc_args a)
{
	constexpr int BSZ = BITS * 4 + 1, G = 4 / CH, GDW = BSZ;
	constexpr int IN = 64 * 256;		/* PCM bytes per wave */
	constexpr int NOUT = 64 * GDW * 4;	/* XA bytes per wave */
	__shared__ __attribute__((aligned(16))) uint8_t lds[XA_ENC_WPB * IN];
	const int lane = threadIdx.x & 63;
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	uint8_t *buf = lds + wv * IN;
	const uint64_t grp0 = ((uint64_t)blockIdx.x * XA_ENC_WPB + wv) * 64u;
	const uint64_t ngroups = ((uint64_t)a.eblocks + G - 1) / G;
	if (grp0 >= ngroups)
		return;
	const uint64_t pcm_bytes = a.frames * CH * 2u;
	const uint64_t base = grp0 * 256u;		/* wave's first PCM byte */
	const bool full = base + IN <= pcm_bytes;

	/* stage: DMA instruction i, lane t fills position t % 16 of row
	 * 4i + t / 16 with piece (t % 16) ^ (row & 15) of that row */
	const uint64_t lastp = (pcm_bytes - 1) & ~(uint64_t)15;
	/* wave priority: a starting wave issues its DMA ahead of the other
	 * waves' packing VALU (2), its stores next (1): 168.0 -> 166.2 us on
	 * C3-shaped PCM, one box */
	__builtin_amdgcn_s_setprio(2);
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const int row = 4 * i + (lane >> 4);
		const int piece = (lane & 15) ^ (row & 15);
		uint64_t off = base + (uint64_t)row * 256u + piece * 16u;
		if (!full && off > lastp)
			off = lastp;	/* past the end: any valid piece */
		__builtin_amdgcn_global_load_lds(a.src + off, LDS_PTR(buf + i * 1024),
		    16, 0, 0);
	}
	__builtin_amdgcn_s_setprio(0);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	wave_sync();

	uint32_t pcm[64];
	const uint8_t *row = buf + lane * 256;
#pragma unroll
	for (int j = 0; j < 16; j++) {
		const u32x4a v = *(const u32x4a *)(row + 16 * (j ^ (lane & 15)));
		pcm[4 * j] = v.x;
		pcm[4 * j + 1] = v.y;
		pcm[4 * j + 2] = v.z;
		pcm[4 * j + 3] = v.w;
	}
	if (!full) {
		/* frames past the end encode as 0 (src/libbjxa.c:686-690) */
		const uint64_t g0 = base + (uint64_t)lane * 256u;
#pragma unroll
		for (int d = 0; d < 64; d++) {
			const uint64_t o = g0 + 4u * d;
			const uint32_t lo = o < pcm_bytes ? 0xffffu : 0u;
			const uint32_t hi = o + 2u < pcm_bytes ? 0xffff0000u : 0u;
			pcm[d] &= lo | hi;
		}
	}
	wave_sync();

	uint32_t *obuf = (uint32_t *)buf;
#pragma unroll
	for (int d = 0; d < GDW; d++)
		obuf[lane * GDW + d] = enc_byte<BITS, CH>(pcm, 4 * d) |
		    (enc_byte<BITS, CH>(pcm, 4 * d + 1) << 8) |
		    (enc_byte<BITS, CH>(pcm, 4 * d + 2) << 16) |
		    (enc_byte<BITS, CH>(pcm, 4 * d + 3) << 24);
	wave_sync();

	/* the wave's XA run: groups past the last eblock are not written */
	const uint64_t nxa = (uint64_t)a.eblocks * CH * BSZ;
	const uint64_t ostart = grp0 * 4u * BSZ;
	uint8_t *dst = a.dst + ostart;
	const uint64_t valid = nxa - ostart < (uint64_t)NOUT ? nxa - ostart :
	    (uint64_t)NOUT;
	if (valid == (uint64_t)NOUT && ((uintptr_t)dst & 15u) == 0) {
		__builtin_amdgcn_s_setprio(1);
#pragma unroll
		for (int i = 0; i < (NOUT / 16 + 63) / 64; i++) {
			const int k = 64 * i + lane;
			if (k < NOUT / 16)
				__builtin_nontemporal_store(
				    *(const u32x4a *)(buf + 16 * k),
				    (u32x4a *)(dst + 16 * k));
		}
		return;
	}
	for (uint32_t k = lane; 4u * k < valid; k += 64u) {
		const uint32_t v = obuf[k];
		if (4u * k + 4u <= valid) {
			*(uint32_t *)(dst + 4u * k) = v;
		} else {
			for (uint32_t q = 0; 4u * k + q < valid; q++)
				dst[4u * k + q] = (uint8_t)(v >> (8 * q));
		}
	}
}

hipError_t
xa_encode_launch(const xa_enc_args &a, unsigned bits, unsigned ch,
    hipStream_t st)
{
	const uint64_t G = 4 / ch;
	const uint64_t ngroups = ((uint64_t)a.eblocks + G - 1) / G;
	const uint64_t nwaves = (ngroups + 63) / 64;
	const unsigned grid = (unsigned)((nwaves + XA_ENC_WPB - 1) / XA_ENC_WPB);
	if (grid == 0)
		return hipSuccess;
#define L(B, C) hipLaunchKernelGGL((xa_encode_waves<B, C>), dim3(grid), \
    dim3(64 * XA_ENC_WPB), 0, st, a)
	if (ch == 1) {
		if (bits == 8) L(8, 1); else if (bits == 6) L(6, 1); else L(4, 1);
	} else {
		if (bits == 8) L(8, 2); else if (bits == 6) L(6, 2); else L(4, 2);
	}
#undef L
	return hipGetLastError();
}
