/*
 * xa_small.hip -- low-latency path for small host-API calls.
 *
 * A bjxa_decode()/bjxa_encode() call on a few blocks (the reference CLI's
 * default loop makes one call per block, src/bjxa_decode.c:102-155,
 * src/bjxa_encode.c:112-165) is bound by round trips, not bandwidth.  These
 * kernels take their input from, and leave their output and status in, the
 * codec's pinned host buffer (device-mapped), so a call is one memcpy into
 * that buffer, one single-workgroup launch, one stream sync and one memcpy
 * out -- no hipMemcpy and no second kernel.
 *
 * Decode: the input is staged into LDS with coalesced reads over PCIe; a
 * pre-pass finds the first channel block whose gain nibble is >= 5
 * (src/libbjxa.c:547-550); then one lane per channel decodes its blocks in
 * order up to that block, with the same xa_step as the main kernels -- so a
 * bad right block leaves the left channel advanced through that eblock, as
 * the reference does (:633-643).  Encode is stateless: one lane per channel
 * block (src/libbjxa.c:665-691, :349-391).
 */
#include "xa_common.h"
#include "xa_decode.h"

/* int16 inflate value of code k of a channel block (src/libbjxa.c:286-345) */
template <int BITS>
__device__ __forceinline__ int32_t
small_code(const uint8_t *blk, int k)
{
	if (BITS == 8)
		return (int32_t)(int16_t)((uint32_t)blk[1 + k] << 8);
	if (BITS == 4) {
		const uint32_t v = blk[1 + k / 2];
		return (int32_t)(int16_t)(((k & 1) ? (v & 15u) : (v >> 4)) << 12);
	}
	const uint8_t *g = blk + 1 + 3 * (k / 4);
	const uint32_t s = ((uint32_t)g[0] << 16) | ((uint32_t)g[1] << 8) | g[2];
	return (int32_t)(int16_t)(((s >> (18 - 6 * (k % 4))) & 63u) << 10);
}

template <int BITS, int CH>
__global__ __launch_bounds__(64) void
xa_decode_small(const uint8_t *in_h, uint8_t *out_h, uint32_t n,
    uint32_t init0, uint32_t init1)
{
	constexpr int BSZ = BITS * 4 + 1, EBSZ = BSZ * CH;
	__shared__ __attribute__((aligned(16))) uint8_t in[XA_SMALL_MAX * EBSZ + 4];
	__shared__ __attribute__((aligned(16))) int16_t pcm[XA_SMALL_MAX * 32 * CH];
	__shared__ uint32_t err;
	const uint32_t t = threadIdx.x;
	const uint32_t nin = n * EBSZ;

	for (uint32_t i = t; i < (nin + 3) / 4; i += 64)
		((uint32_t *)in)[i] = ((const uint32_t *)in_h)[i];
	if (t == 0)
		err = 0xffffffffu;
	__syncthreads();
	if (t < n * CH && (in[t * BSZ] >> 4) >= 5u)
		atomicMin(&err, t);
	__syncthreads();
	if (t < (uint32_t)CH) {
		int32_t p0, p1;
		xa_unpack_state(t ? init1 : init0, p0, p1);
		const uint32_t e = err;
		for (uint32_t b = 0; b < n && b * CH + t < e; b++) {
			const uint8_t *blk = in + (b * CH + t) * BSZ;
			const uint32_t prof = blk[0];
			int32_t k0, k1;
			xa_gain((prof >> 4) & 7u, k0, k1);
			for (int k = 0; k < XA_FRAMES; k++) {
				const int32_t code = small_code<BITS>(blk, k);
				pcm[(b * XA_FRAMES + k) * CH + t] = (int16_t)xa_step(
				    (int32_t)((uint32_t)code << 16), 16u + (prof & 15u),
				    k0, k1, p0, p1);
			}
		}
		uint32_t *st = (uint32_t *)(out_h + XA_SMALL_STATUS);
		st[1 + t] = xa_pack_state(p0, p1);
		if (t == 0) {
			st[0] = e;
			if (CH == 1)
				st[2] = init1;
		}
	}
	__syncthreads();
	for (uint32_t i = t; i < n * 16u * CH; i += 64)
		((uint32_t *)out_h)[i] = ((const uint32_t *)pcm)[i];
}

template <int BITS, int CH>
__global__ __launch_bounds__(64) void
xa_encode_small(const uint8_t *in_h, uint8_t *out_h, uint64_t frames)
{
	constexpr int BSZ = BITS * 4 + 1;
	__shared__ __attribute__((aligned(16))) int16_t pcm[XA_SMALL_MAX * 32 * CH];
	__shared__ __attribute__((aligned(16))) uint8_t xa[XA_SMALL_MAX * BSZ * CH + 4];
	const uint32_t t = threadIdx.x;
	const uint32_t n = (uint32_t)((frames + 31) / 32);
	const uint32_t nsmp = (uint32_t)frames * CH;

	/* frames past the end encode as 0 (src/libbjxa.c:686-690) */
	for (uint32_t i = t; i < n * 32u * CH; i += 64)
		pcm[i] = i < nsmp ? ((const int16_t *)in_h)[i] : (int16_t)0;
	__syncthreads();
	if (t < n * CH) {
		const uint32_t b = t / CH, c = t % CH;
		uint8_t *blk = xa + t * BSZ;
#define S(k) ((uint32_t)(uint16_t)pcm[(b * XA_FRAMES + (k)) * CH + c])
		blk[0] = 0;		/* profile (src/libbjxa.c:679) */
		for (int j = 0; j < BSZ - 1; j++) {
			uint32_t v;
			if (BITS == 8) {
				v = S(j) >> 8;
			} else if (BITS == 4) {
				v = ((S(2 * j) >> 8) & 0xf0u) | (S(2 * j + 1) >> 12);
			} else {
				const int g = j / 3, r = j % 3;
				const uint32_t s24 = ((S(4 * g) >> 10) << 18) |
				    ((S(4 * g + 1) >> 10) << 12) |
				    ((S(4 * g + 2) >> 10) << 6) | (S(4 * g + 3) >> 10);
				v = s24 >> (16 - 8 * r);
			}
			blk[1 + j] = (uint8_t)v;
		}
#undef S
	}
	__syncthreads();
	const uint32_t nb = n * BSZ * CH;
	for (uint32_t i = t; i < nb; i += 64)
		out_h[i] = xa[i];
}

hipError_t
xa_small_decode_launch(const uint8_t *in_h, uint8_t *out_h, uint32_t n,
    unsigned bits, unsigned ch, const uint32_t init[2], hipStream_t st)
{
#define L(B, C) hipLaunchKernelGGL((xa_decode_small<B, C>), dim3(1), dim3(64), \
    0, st, in_h, out_h, n, init[0], init[1])
	if (ch == 1) {
		if (bits == 8) L(8, 1); else if (bits == 6) L(6, 1); else L(4, 1);
	} else {
		if (bits == 8) L(8, 2); else if (bits == 6) L(6, 2); else L(4, 2);
	}
#undef L
	return hipGetLastError();
}

hipError_t
xa_small_encode_launch(const uint8_t *in_h, uint8_t *out_h, uint64_t frames,
    unsigned bits, unsigned ch, hipStream_t st)
{
#define L(B, C) hipLaunchKernelGGL((xa_encode_small<B, C>), dim3(1), dim3(64), \
    0, st, in_h, out_h, frames)
	if (ch == 1) {
		if (bits == 8) L(8, 1); else if (bits == 6) L(6, 1); else L(4, 1);
	} else {
		if (bits == 8) L(8, 2); else if (bits == 6) L(6, 2); else L(4, 2);
	}
#undef L
	return hipGetLastError();
}
