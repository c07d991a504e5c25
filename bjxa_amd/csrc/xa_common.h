/*
 * xa_common.h -- block geometry and arithmetic shared by the gfx950 kernels.
 *
 * Format facts (reference src/libbjxa.c):
 *   channel block = 1 profile byte + bits*4 data bytes            (:431)
 *   effective block (eblock) = L block [+ R block], 32 frames     (:629-646)
 *   profile = gain<<4 | range; gain >= 5 is a protocol error      (:547-550)
 *   K0/K1 x 256 per gain                                          (:525-531)
 */
#ifndef BJXA_XA_COMMON_H
#define BJXA_XA_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define XA_FRAMES 32

/* channel block / effective block sizes in bytes */
template <int BITS> struct xa_bits {
	static constexpr int BSZ = BITS * 4 + 1;
	/* a "group" is 4 channel blocks (4 mono blocks or 2 stereo eblocks):
	 * 4*BSZ bytes = BSZ dwords, always 4-byte aligned */
	static constexpr int GDW = BSZ;
};

/*
 * K0 (9 bits, unsigned) and |K1| (8 bits) packed per gain so a lane can pick
 * its block's pair with two shifts instead of a table load.  Gains 5-7 (the
 * error case) map to 0/0; their output is never emitted.
 */
__device__ __forceinline__ void
xa_gain(uint32_t gain, int32_t &k0, int32_t &k1)
{
	const uint64_t K0 = (0ull) | (240ull << 9) | (460ull << 18) |
	    (392ull << 27) | (488ull << 36);
	const uint64_t K1 = (0ull) | (0ull << 8) | (208ull << 16) |
	    (220ull << 24) | (240ull << 32);
	k0 = (int32_t)((K0 >> (gain * 9)) & 511u);
	k1 = -(int32_t)((K1 >> (gain * 8)) & 255u);
}

/*
 * One predictor step (src/libbjxa.c:556-572):
 *   s = clamp(t + trunc((p0*K0 + p1*K1) / 256))
 * `top` holds the unpacked code left-justified at bit 31 with zeros below
 * bit 16, so t = top >> (16 + range) equals (int16 code) >> range.
 * The truncating divide is floor((g + 255*[g<0]) / 256).
 */
__device__ __forceinline__ int32_t
xa_step(int32_t top, uint32_t sh, int32_t k0, int32_t k1, int32_t &p0,
    int32_t &p1)
{
	int32_t t = top >> sh;
	int32_t g = __mul24(p0, k0) + __mul24(p1, k1);
	int32_t s = t + ((g + (int32_t)((uint32_t)(g >> 31) >> 24)) >> 8);
	s = min(max(s, -32768), 32767);
	p1 = p0;
	p0 = s;
	return s;
}

/*
 * Both channels of one stereo frame in one instruction stream, on the
 * packed-f32 pipe (the two chains ride the two halves of v_pk_fma_f32):
 *
 *   g    = p0 * K0/256 + p1 * K1/256          v_pk_mul_f32 + v_pk_fma_f32
 *   q    = trunc(g)                           v_cvt_i32_f32 x2
 *   s    = q + t                              v_add_u32_sdwa (sext t) x2
 *   out  = sat16(s) packed L | R << 16        v_cvt_pk_i16_i32
 *   p0'  = float(out.lo), float(out.hi)       v_cvt_f32_i32_sdwa x2
 *
 * Exactness: p0, p1 are int16 and |K0| <= 488, |K1| <= 240, so each product
 * is exact in f32 (|p*K| < 2^24) and the fma rounds once; the sum is exact
 * while |g*256| < 2^24.  Beyond that |q| >= 65536 both before and after
 * rounding, so s saturates to the same int16 either way.  v_cvt_i32_f32
 * truncates toward zero, which is the reference's `/ 256` on int
 * (src/libbjxa.c:565-566), and v_cvt_pk_i16_i32 saturates as its clamp
 * (:567-570).
 *
 * `t` holds the two int16 inflate values already shifted by range (low half
 * L, high half R).  Returns the frame; p0/p1 advance.
 */
typedef float xa_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t
xa_step_lr(uint32_t t, xa_f2 k0, xa_f2 k1, xa_f2 &p0, xa_f2 &p1)
{
	const xa_f2 g = __builtin_elementwise_fma(p0, k0, p1 * k1);
	const int32_t sl = (int32_t)g.x + (int32_t)(int16_t)(t & 0xffffu);
	const int32_t sr = (int32_t)g.y + (int32_t)(int16_t)(t >> 16);
	typedef short xa_s2 __attribute__((ext_vector_type(2)));
	const xa_s2 pk = __builtin_amdgcn_cvt_pk_i16(sl, sr);
	const uint32_t fr = __builtin_bit_cast(uint32_t, pk);
	const float fl = (float)(int16_t)(fr & 0xffffu);
	const float fh = (float)(int16_t)(fr >> 16);
	p1 = p0;
	p0 = xa_f2{fl, fh};
	return fr;
}

/*
 * One channel's step with the same f32 prediction (mono: one chain per
 * lane, nothing to pack).  `th` is the int16 inflate value, shifted by
 * range, in the low (HI = false) or high half of t:
 *   v_pk_mul_f32/v_mul_f32 + v_fma_f32, v_cvt_i32_f32, v_add_u32_sdwa
 *   (sext), v_med3_i32, v_cvt_f32_i32 -- 5 dependent operations, against
 *   the integer step's 6 plus its separate range shift.
 * Exactness as xa_step_lr; the clamp is explicit here.
 */
template <bool HI>
__device__ __forceinline__ int32_t
xa_step_f(uint32_t t, float k0, float k1, float &p0, float &p1)
{
	const float g = __builtin_fmaf(p0, k0, p1 * k1);
	int32_t s = (int32_t)g + (int32_t)(int16_t)(HI ? t >> 16 : t & 0xffffu);
	s = min(max(s, -32768), 32767);
	p1 = p0;
	p0 = (float)s;
	return s;
}

/* per-channel K pair of a gain as the f32 factors of xa_step_lr */
__device__ __forceinline__ void
xa_gain_f(uint32_t gain, float &k0, float &k1)
{
	int32_t a, b;
	xa_gain(gain, a, b);
	k0 = (float)a * (1.0f / 256.0f);
	k1 = (float)b * (1.0f / 256.0f);
}

/* two int16 values shifted right arithmetically, each by its own count
 * (v_pk_ashrrev_i16: low half by sh's low half, high by its high half) */
__device__ __forceinline__ uint32_t
xa_pk_ashr(uint32_t v, uint32_t sh)
{
	uint32_t r;
	asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(r) : "v"(sh), "v"(v));
	return r;
}

/*
 * The helpers below take byte/code indices as plain ints: every call site
 * sits inside fully unrolled loops, so the indices fold to constants and
 * w[] stays in VGPRs (checked: no scratch in the kernel resource usage).
 */

/* byte b of the dword array, moved to bits 24..31, zeros below */
__device__ __forceinline__ uint32_t
xa_byte_top(const uint32_t *w, const int b)
{
	return __builtin_amdgcn_perm(0u, w[b >> 2], 0x000c0c0cu |
	    ((uint32_t)(b & 3) << 24));
}

/* bytes b (-> bits 24..31) and b+1 (-> bits 16..23) */
__device__ __forceinline__ uint32_t
xa_2bytes_top(const uint32_t *w, const int b)
{
	if ((b >> 2) == ((b + 1) >> 2)) {
		return __builtin_amdgcn_perm(0u, w[b >> 2], 0x00000c0cu |
		    ((uint32_t)(b & 3) << 24) | ((uint32_t)((b + 1) & 3) << 16));
	}
	/* b is byte 3 of w[i], b+1 is byte 0 of w[i+1]; v_perm_b32 indexes
	 * the 64-bit {S0, S1}: selectors 0-3 pick bytes of S1 (w[i]),
	 * 4-7 bytes of S0 (w[i+1]) */
	return __builtin_amdgcn_perm(w[(b + 1) >> 2], w[b >> 2],
	    0x00000c0cu | (3u << 24) | (4u << 16));
}

/*
 * Code n (0..31) of the channel block whose profile byte is byte o of w,
 * left-justified: bits 31..16 hold the reference's int16 inflate value
 * (src/libbjxa.c:286-345), lower bits are zero.
 */
template <int BITS>
__device__ __forceinline__ int32_t
code_at(const uint32_t *w, const int o, const int n)
{
	if (BITS == 8)
		return (int32_t)xa_byte_top(w, o + 1 + n);
	if (BITS == 4) {
		/* high nibble first (src/libbjxa.c:295-298) */
		uint32_t v = xa_byte_top(w, o + 1 + n / 2);
		return (int32_t)((n & 1) ? (v << 4) : (v & 0xf0000000u));
	}
	/* 6-bit: 4 codes per 3 bytes, big-endian (src/libbjxa.c:315-321) */
	const int bit = 6 * n, byte = bit >> 3, off = bit & 7;
	uint32_t v = off <= 2 ? xa_byte_top(w, o + 1 + byte) :
	    xa_2bytes_top(w, o + 1 + byte);
	return (int32_t)((v << off) & 0xfc000000u);
}

/* state word: p0 in bits 0..15, p1 in bits 16..31 */
__device__ __forceinline__ uint32_t
xa_pack_state(int32_t p0, int32_t p1)
{
	return ((uint32_t)p0 & 0xffffu) | ((uint32_t)p1 << 16);
}

__device__ __forceinline__ void
xa_unpack_state(uint32_t s, int32_t &p0, int32_t &p1)
{
	p0 = (int32_t)(int16_t)(s & 0xffffu);
	p1 = (int32_t)(int16_t)(s >> 16);
}

#endif
