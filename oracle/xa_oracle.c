/*
 * xa_oracle.c -- CPU restatement of libbjxa's XA ADPCM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Nothing in bjxa_amd/ links, loads or calls it; the product path runs on
 * the GPU and fails loudly without it.
 *
 * Written from the format contract (bjxa.5.rst), not from
 * the reference source text.  Each routine names the reference routine whose
 * behaviour it restates (paths relative to the reference checkout).
 *
 * Pinning: the reference cannot be built in this image without a stand-in
 * for its autoconf-generated config.h, so there is no oracle/_ref.  The
 * restatement is pinned by the reference's own known-answer tests instead:
 * the six decode SHA-1s and the saturation vector of test/test_decode.sh
 * (:24-122), checked by tests/test_oracle.py.
 */

#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define XO_SAMPLES 32

/* K0/K1 x 256 per gain nibble; src/libbjxa.c:525-531. */
static const int32_t xo_k[5][2] = {
	{ 0, 0 }, { 240, 0 }, { 460, -208 }, { 392, -220 }, { 488, -240 },
};

/*
 * Unpack one block's 32 codes into left-justified int16.
 * 4-bit: src/libbjxa.c:286-302 (high nibble first),
 * 6-bit: src/libbjxa.c:304-327 (big-endian 24-bit groups of 4 codes),
 * 8-bit: src/libbjxa.c:329-345.
 */
static void
xo_unpack(int16_t out[XO_SAMPLES], const uint8_t *data, unsigned bits)
{
	unsigned i;

	if (bits == 8) {
		for (i = 0; i < XO_SAMPLES; i++)
			out[i] = (int16_t)(uint16_t)(data[i] << 8);
	} else if (bits == 4) {
		for (i = 0; i < XO_SAMPLES / 2; i++) {
			out[2 * i] = (int16_t)(uint16_t)((data[i] & 0xf0u) << 8);
			out[2 * i + 1] = (int16_t)(uint16_t)((data[i] & 0x0fu) << 12);
		}
	} else {
		for (i = 0; i < XO_SAMPLES / 4; i++) {
			uint32_t g = ((uint32_t)data[3 * i] << 16) |
			    ((uint32_t)data[3 * i + 1] << 8) | data[3 * i + 2];
			unsigned j;
			for (j = 0; j < 4; j++) {
				uint32_t code = (g >> (18 - 6 * j)) & 63u;
				out[4 * i + j] = (int16_t)(uint16_t)(code << 10);
			}
		}
	}
}

/*
 * Two-tap predictor over one block; src/libbjxa.c:533-578.
 * Returns -1 for a gain nibble >= 5 (the reference's EPROTO at :550).
 */
static int
xo_predict(int16_t x[XO_SAMPLES], uint8_t profile, int16_t st[2])
{
	unsigned f = profile >> 4, r = profile & 15u, i;
	int32_t p0 = st[0], p1 = st[1];

	if (f >= 5)
		return (-1);
	for (i = 0; i < XO_SAMPLES; i++) {
		int32_t t = (int32_t)x[i] >> r;
		int32_t g = p0 * xo_k[f][0] + p1 * xo_k[f][1];
		int32_t s = t + g / 256;	/* C division truncates */
		if (s < -32768)
			s = -32768;
		if (s > 32767)
			s = 32767;
		x[i] = (int16_t)s;
		p1 = p0;
		p0 = s;
	}
	st[0] = (int16_t)p0;
	st[1] = (int16_t)p1;
	return (0);
}

/*
 * Single-pass decode of `eblocks` effective blocks (bjxa_decode,
 * src/libbjxa.c:602-661, called once for a whole stream).
 *
 * state[0..1] = left prev[0..1], state[2..3] = right prev[0..1]; updated.
 * pcm receives min(32, frames left) frames per block, channels interleaved.
 * Returns the number of effective blocks fully decoded.  When a bad profile
 * stops the loop, *bad_chan names the failing channel (else -1) and the
 * state reflects the reference's partial update: a bad right block leaves
 * the left channel already advanced over that frame.
 */
uint64_t
xo_decode(const uint8_t *xa, uint64_t eblocks, unsigned bits, unsigned ch,
    int16_t state[4], int16_t *pcm, uint64_t frames, int *bad_chan)
{
	unsigned bsz = bits * 4 + 1;
	uint64_t b, left = frames;
	int16_t buf[2][XO_SAMPLES];

	*bad_chan = -1;
	for (b = 0; b < eblocks; b++) {
		unsigned c, n, take;
		for (c = 0; c < ch; c++) {
			const uint8_t *blk = xa + (b * ch + c) * bsz;
			xo_unpack(buf[c], blk + 1, bits);
			if (xo_predict(buf[c], blk[0], state + 2 * c) < 0) {
				*bad_chan = (int)c;
				return (b);
			}
		}
		take = left < XO_SAMPLES ? (unsigned)left : XO_SAMPLES;
		for (n = 0; n < take; n++)
			for (c = 0; c < ch; c++)
				pcm[n * ch + c] = buf[c][n];
		pcm += (size_t)take * ch;
		left -= take;
	}
	return (eblocks);
}

/*
 * Pack one channel's block; src/libbjxa.c:349-391 (the inverse of unpack:
 * keep the top `bits` bits of each sample as an unsigned 16-bit value).
 */
static void
xo_pack(uint8_t *data, const int16_t in[XO_SAMPLES], unsigned bits)
{
	unsigned i;

	if (bits == 8) {
		for (i = 0; i < XO_SAMPLES; i++)
			data[i] = (uint8_t)((uint16_t)in[i] >> 8);
	} else if (bits == 4) {
		for (i = 0; i < XO_SAMPLES / 2; i++)
			data[i] = (uint8_t)((((uint16_t)in[2 * i] >> 12) << 4) |
			    ((uint16_t)in[2 * i + 1] >> 12));
	} else {
		for (i = 0; i < XO_SAMPLES / 4; i++) {
			uint32_t g = 0;
			unsigned j;
			for (j = 0; j < 4; j++)
				g |= (uint32_t)((uint16_t)in[4 * i + j] >> 10) <<
				    (18 - 6 * j);
			data[3 * i] = (uint8_t)(g >> 16);
			data[3 * i + 1] = (uint8_t)(g >> 8);
			data[3 * i + 2] = (uint8_t)g;
		}
	}
}

/*
 * Single-pass encode of `frames` frames (bjxa_encode, src/libbjxa.c:759-819
 * with bjxa_encode_inflated :665-691): profile byte 0, the partial last
 * block zero-padded.  Writes ceil(frames/32) effective blocks.
 */
uint64_t
xo_encode(const int16_t *pcm, uint64_t frames, unsigned bits, unsigned ch,
    uint8_t *xa)
{
	unsigned bsz = bits * 4 + 1;
	uint64_t b, eblocks = (frames + XO_SAMPLES - 1) / XO_SAMPLES;
	int16_t buf[XO_SAMPLES];

	for (b = 0; b < eblocks; b++) {
		uint64_t f0 = b * XO_SAMPLES;
		unsigned c, n, take = (unsigned)((frames - f0) < XO_SAMPLES ?
		    (frames - f0) : XO_SAMPLES);
		for (c = 0; c < ch; c++) {
			uint8_t *blk = xa + (b * ch + c) * bsz;
			for (n = 0; n < XO_SAMPLES; n++)
				buf[n] = n < take ? pcm[(f0 + n) * ch + c] : 0;
			blk[0] = 0;
			xo_pack(blk + 1, buf, bits);
		}
	}
	return (eblocks);
}
