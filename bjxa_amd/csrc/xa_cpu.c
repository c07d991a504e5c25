/*
 * xa_cpu.c -- the CPU core of libbjxa.so.0.
 *
 * bjxa_decode()/bjxa_encode() run here when a call is too small to pay for
 * a GPU round trip (the reference CLI's default loop makes one call per
 * block, src/bjxa_decode.c:122-152) and on hosts without a GPU.  Larger
 * calls go to the gfx950 kernels (xa_gpu.hip); libbjxa.c picks the side
 * with bjxa__offload().
 *
 * The arithmetic is the reference's (src/libbjxa.c):
 *   unpack 4/6/8-bit codes left-justified into int16     (:286-345)
 *   t = code >> range; s = clamp(t + trunc((p0*K0 + p1*K1) / 256))
 *   p1 = p0; p0 = s, per channel, across every block     (:533-578)
 *   encode: profile 0, top `bits` bits of each sample    (:349-391, :665-691)
 * but the loop is shaped for a core rather than restated: the codes of a
 * block are unpacked and range-shifted in one pass, and a stereo eblock
 * runs its left and right predictor chains in the same loop so the two
 * independent dependency chains overlap in the core's pipelines (the
 * reference decodes the left block, then the right one, :633-646).
 */
#include <stdint.h>
#include <string.h>

#include "xa_gpu.h"

#define FRAMES	32

/* gain_factor x 256 (src/libbjxa.c:525-531): K0, K1 per gain nibble */
static const int32_t k_gain[5][2] = {
	{ 0, 0 }, { 240, 0 }, { 460, -208 }, { 392, -220 }, { 488, -240 },
};

/*
 * The 32 codes of one channel block as int32, already shifted by the
 * block's range: (int16)(code << (16 - bits)) >> range.  A left-justified
 * int16 code c<<8 is (int8)c * 256, so no int16 wrap is needed.
 */
static void
unpack(const uint8_t *blk, unsigned bits, int32_t t[FRAMES])
{
	const unsigned r = blk[0] & 15u;
	const uint8_t *d = blk + 1;
	int i;

	switch (bits) {
	case 8:
		for (i = 0; i < FRAMES; i++)
			t[i] = ((int32_t)(int8_t)d[i] * 256) >> r;
		break;
	case 6:
		for (i = 0; i < FRAMES / 4; i++) {
			const uint32_t s = (uint32_t)d[3 * i] << 16 |
			    (uint32_t)d[3 * i + 1] << 8 | d[3 * i + 2];
			t[4 * i] = ((int32_t)(int8_t)((s >> 16) & 0xfcu) *
			    256) >> r;
			t[4 * i + 1] = ((int32_t)(int8_t)((s >> 10) & 0xfcu) *
			    256) >> r;
			t[4 * i + 2] = ((int32_t)(int8_t)((s >> 4) & 0xfcu) *
			    256) >> r;
			t[4 * i + 3] = ((int32_t)(int8_t)((s << 2) & 0xfcu) *
			    256) >> r;
		}
		break;
	default:	/* 4 */
		for (i = 0; i < FRAMES / 2; i++) {
			t[2 * i] = ((int32_t)(int8_t)(d[i] & 0xf0u) * 256) >> r;
			t[2 * i + 1] = ((int32_t)(int8_t)(d[i] << 4) * 256) >> r;
		}
		break;
	}
}

static inline int32_t
clamp16(int32_t s)
{
	return s < -32768 ? -32768 : s > 32767 ? 32767 : s;
}

/* one channel block through the predictor, output at stride `ch` */
static void
run_block(const int32_t t[FRAMES], unsigned gain, int16_t *st, int16_t *out,
    unsigned ch)
{
	const int32_t k0 = k_gain[gain][0], k1 = k_gain[gain][1];
	int32_t p0 = st[0], p1 = st[1];
	int i;

	for (i = 0; i < FRAMES; i++) {
		const int32_t s = clamp16(t[i] + (p0 * k0 + p1 * k1) / 256);
		p1 = p0;
		p0 = s;
		out[i * ch] = (int16_t)s;
	}
	st[0] = (int16_t)p0;
	st[1] = (int16_t)p1;
}

/* both blocks of a stereo eblock, the two chains interleaved */
static void
run_pair(const int32_t tl[FRAMES], const int32_t tr[FRAMES], unsigned gl,
    unsigned gr, int16_t st[4], int16_t out[2 * FRAMES])
{
	const int32_t a0 = k_gain[gl][0], a1 = k_gain[gl][1];
	const int32_t b0 = k_gain[gr][0], b1 = k_gain[gr][1];
	int32_t l0 = st[0], l1 = st[1], r0 = st[2], r1 = st[3];
	int i;

	for (i = 0; i < FRAMES; i++) {
		const int32_t sl = clamp16(tl[i] + (l0 * a0 + l1 * a1) / 256);
		const int32_t sr = clamp16(tr[i] + (r0 * b0 + r1 * b1) / 256);
		l1 = l0;
		l0 = sl;
		r1 = r0;
		r0 = sr;
		out[2 * i] = (int16_t)sl;
		out[2 * i + 1] = (int16_t)sr;
	}
	st[0] = (int16_t)l0;
	st[1] = (int16_t)l1;
	st[2] = (int16_t)r0;
	st[3] = (int16_t)r1;
}

/*
 * Same contract as bjxa__gpu_decode (xa_gpu.h): decode `eblocks` eblocks
 * of `src` from `state`, copy the first `dst_bytes` PCM bytes to `dst`,
 * stop before the first eblock holding a channel block whose gain nibble
 * is >= 5 (*err_cb = its channel block index; for a bad right block the
 * left channel of that eblock is advanced, as the reference's per-channel
 * loop leaves it, :633-646).
 */
int
bjxa__cpu_decode(const void *src, uint32_t eblocks, unsigned bits,
    unsigned ch, int16_t state[4], void *dst, uint64_t dst_bytes,
    uint32_t *err_cb)
{
	const uint8_t *in = src;
	uint8_t *out = dst;
	const unsigned bsz = bits * 4 + 1, pcm = 2u * FRAMES * ch;
	int32_t tl[FRAMES], tr[FRAMES];
	int16_t frame[2 * FRAMES];
	uint32_t b;

	*err_cb = 0xffffffffu;
	for (b = 0; b < eblocks; b++, in += bsz * ch) {
		const unsigned gl = in[0] >> 4;

		if (gl >= 5) {
			*err_cb = b * ch;
			return 0;
		}
		unpack(in, bits, tl);
		if (ch == 1) {
			run_block(tl, gl, state, frame, 1);
		} else {
			const unsigned gr = in[bsz] >> 4;
			if (gr >= 5) {
				/* the left block runs before the right one
				 * is found bad (:633-643) */
				run_block(tl, gl, state, frame, 2);
				*err_cb = b * 2 + 1;
				return 0;
			}
			unpack(in + bsz, bits, tr);
			run_pair(tl, tr, gl, gr, state, frame);
		}
		if (dst_bytes >= pcm) {
			memcpy(out, frame, pcm);
			out += pcm;
			dst_bytes -= pcm;
		} else if (dst_bytes > 0) {
			memcpy(out, frame, (size_t)dst_bytes);
			out += dst_bytes;
			dst_bytes = 0;
		}
	}
	return 0;
}

/* pack the top `bits` bits of 32 samples (src/libbjxa.c:349-391) */
static void
pack(const uint16_t s[FRAMES], unsigned bits, uint8_t *d)
{
	int i;

	switch (bits) {
	case 8:
		for (i = 0; i < FRAMES; i++)
			d[i] = (uint8_t)(s[i] >> 8);
		break;
	case 6:
		for (i = 0; i < FRAMES / 4; i++) {
			const uint32_t v = (uint32_t)(s[4 * i] >> 10) << 18 |
			    (uint32_t)(s[4 * i + 1] >> 10) << 12 |
			    (uint32_t)(s[4 * i + 2] >> 10) << 6 |
			    (uint32_t)(s[4 * i + 3] >> 10);
			d[3 * i] = (uint8_t)(v >> 16);
			d[3 * i + 1] = (uint8_t)(v >> 8);
			d[3 * i + 2] = (uint8_t)v;
		}
		break;
	default:	/* 4 */
		for (i = 0; i < FRAMES / 2; i++)
			d[i] = (uint8_t)((s[2 * i] >> 8 & 0xf0u) |
			    s[2 * i + 1] >> 12);
		break;
	}
}

/*
 * Same contract as bjxa__gpu_encode: `frames` frames of host-order int16
 * PCM into ceil(frames / 32) eblocks, profile 0, the last block padded with
 * zero samples (:686-690).
 */
int
bjxa__cpu_encode(const void *src, uint64_t frames, unsigned bits, unsigned ch,
    void *dst)
{
	const uint8_t *in = src;
	uint8_t *out = dst;
	const unsigned bsz = bits * 4 + 1;
	uint16_t pcm[2 * FRAMES], chan[FRAMES];

	while (frames > 0) {
		const unsigned n = frames < FRAMES ? (unsigned)frames : FRAMES;
		unsigned c, i;

		if (n < FRAMES)
			memset(pcm, 0, sizeof pcm);
		memcpy(pcm, in, (size_t)n * 2u * ch);
		for (c = 0; c < ch; c++) {
			for (i = 0; i < FRAMES; i++)
				chan[i] = pcm[i * ch + c];
			out[0] = 0;	/* profile (:679) */
			pack(chan, bits, out + 1);
			out += bsz;
		}
		in += (size_t)n * 2u * ch;
		frames -= n;
	}
	return 0;
}
