/*
 * oracle_drive.c -- command-line driver of oracle/xa_oracle.c for the
 * sanitizer build (make -C bjxa_amd/csrc sanitize, tests/test_sanitize.py).
 * Test infrastructure only.
 *
 *   oracle_drive decode BITS CH FRAMES S0 S1 S2 S3 < blocks > pcm
 *   oracle_drive encode BITS CH FRAMES < pcm > blocks
 *
 * decode: the XA block data (no header), entry state S0..S3; writes the
 * PCM of the whole blocks decoded before any bad profile (at most FRAMES
 * frames) and exits 3 if a profile stopped the loop.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

uint64_t xo_decode(const uint8_t *xa, uint64_t eblocks, unsigned bits,
    unsigned ch, int16_t state[4], int16_t *pcm, uint64_t frames,
    int *bad_chan);
uint64_t xo_encode(const int16_t *pcm, uint64_t frames, unsigned bits,
    unsigned ch, uint8_t *xa);

static uint8_t *
slurp(size_t *len)
{
	size_t cap = 1 << 16, n = 0, r;
	uint8_t *b = malloc(cap);

	while (b != NULL && (r = fread(b + n, 1, cap - n, stdin)) > 0) {
		n += r;
		if (n == cap) {
			uint8_t *nb = realloc(b, cap *= 2);
			if (nb == NULL)
				free(b);
			b = nb;
		}
	}
	*len = n;
	return (b);
}

int
main(int argc, char **argv)
{
	size_t len;
	uint8_t *in;
	unsigned bits, ch;
	uint64_t frames;

	if (argc < 5)
		return (2);
	bits = (unsigned)atoi(argv[2]);
	ch = (unsigned)atoi(argv[3]);
	frames = strtoull(argv[4], NULL, 10);
	if ((bits != 4 && bits != 6 && bits != 8) || (ch != 1 && ch != 2) ||
	    (in = slurp(&len)) == NULL)
		return (2);
	if (strcmp(argv[1], "decode") == 0 && argc == 9) {
		const size_t ebsz = (size_t)(bits * 4 + 1) * ch;
		const uint64_t eb = len / ebsz;
		int16_t st[4], *pcm;
		int bad;
		uint64_t done, n;

		for (int i = 0; i < 4; i++)
			st[i] = (int16_t)atoi(argv[5 + i]);
		if (frames > eb * 32)
			frames = eb * 32;
		pcm = calloc(eb * 32 * ch + 1, sizeof *pcm);
		if (pcm == NULL)
			return (2);
		done = xo_decode(in, eb, bits, ch, st, pcm, frames, &bad);
		n = done * 32 < frames ? done * 32 : frames;
		fwrite(pcm, sizeof *pcm, n * ch, stdout);
		free(pcm);
		free(in);
		return (bad >= 0 ? 3 : 0);
	}
	if (strcmp(argv[1], "encode") == 0 && argc == 5) {
		const uint64_t eb = (frames + 31) / 32;
		const size_t out_len = eb * (bits * 4 + 1) * ch;
		uint8_t *xa;

		if (len < frames * ch * 2)
			return (2);
		xa = malloc(out_len + 1);
		if (xa == NULL)
			return (2);
		xo_encode((const int16_t *)in, frames, bits, ch, xa);
		fwrite(xa, 1, out_len, stdout);
		free(xa);
		free(in);
		return (0);
	}
	return (2);
}
