/*
 * spec_replay.c -- CPU replay of the speculative chunk decode (DESIGN.md
 * §3): for a synthetic stream (8-bit, stereo or mono, a profile mix), cut
 * into chunks of C eblocks with a warm-up of W eblocks from state (0,0),
 * count the chunks whose speculative entry state differs from the true one
 * and how many blocks a repair from the true state runs until it meets the
 * speculative trajectory (cascades: chunks whose repair never meets).
 *
 * build: gcc -O2 -o /tmp/spec_replay tools/spec_replay.c
 * usage: spec_replay <ch> <mix A|F|W> <eblocks> <C> <W>...
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const int K[5][2] = { {0,0}, {240,0}, {460,-208}, {392,-220}, {488,-240} };
static uint64_t s = 0x1234567;

static uint32_t
rnd(void)
{
	s ^= s << 13; s ^= s >> 7; s ^= s << 17;
	return (uint32_t)(s >> 11);
}

/* one channel block of 8-bit codes from state st; returns 1 if the state
 * at block end equals `want` (when want != NULL) */
static void
block(const uint8_t *b, int st[2])
{
	const int g = b[0] >> 4, r = b[0] & 15;
	int p0 = st[0], p1 = st[1];
	for (int i = 0; i < 32; i++) {
		int t = ((int)(int8_t)b[1 + i] * 256) >> r;
		int v = t + (p0 * K[g][0] + p1 * K[g][1]) / 256;
		v = v < -32768 ? -32768 : v > 32767 ? 32767 : v;
		p1 = p0;
		p0 = v;
	}
	st[0] = p0;
	st[1] = p1;
}

int
main(int argc, char **argv)
{
	const int ch = atoi(argv[1]);
	const char mix = argv[2][0];
	const long E = atol(argv[3]), C = atol(argv[4]);
	const long ncb = E * ch;
	uint8_t *xa = malloc(ncb * 33);
	int (*tru)[2] = malloc(sizeof *tru * (ncb + ch));	/* state at each cblock start */

	for (long i = 0; i < ncb; i++) {
		uint8_t *b = xa + i * 33;
		int g, r;
		for (int k = 1; k < 33; k++)
			b[k] = (uint8_t)rnd();
		if (mix == 'A') { g = rnd() % 5; r = rnd() % 13; }
		else if (mix == 'W') { g = 4; r = 12 + rnd() % 4; }
		else { uint32_t u = rnd() % 100000; g = u < 94900 ? 0 : u < 95560 ? 1 : u < 99995 ? 2 : 3; r = rnd() % 4; }
		b[0] = (uint8_t)(g << 4 | r);
	}
	/* true trajectory, per channel */
	for (int c = 0; c < ch; c++) {
		int st[2] = {0, 0};
		for (long e = 0; e < E; e++) {
			tru[e * ch + c][0] = st[0];
			tru[e * ch + c][1] = st[1];
			block(xa + (e * ch + c) * 33, st);
		}
	}
	for (int a = 5; a < argc; a++) {
		const long W = atol(argv[a]);
		long nch = (E + C - 1) / C, mism = 0, casc = 0, hist[64] = {0}, maxr = 0;
		double sumr = 0;
		for (long q = 1; q < nch; q++) {
			const long s0 = q * C;
			int bad = 0;
			long worst = 0;
			for (int c = 0; c < ch; c++) {
				int sp[2] = {0, 0};
				long w0 = s0 - W < 0 ? 0 : s0 - W;
				for (long e = w0; e < s0; e++)
					block(xa + (e * ch + c) * 33, sp);
				if (sp[0] == tru[s0 * ch + c][0] && sp[1] == tru[s0 * ch + c][1])
					continue;
				bad = 1;
				/* repair: blocks until the speculative trajectory meets the
				 * true one at a block end */
				long n = 0;
				for (long e = s0; e < E && e < s0 + C; e++) {
					block(xa + (e * ch + c) * 33, sp);
					n++;
					if (sp[0] == tru[(e + 1) * ch + c][0] && sp[1] == tru[(e + 1) * ch + c][1])
						break;
					if (e + 1 == s0 + C) { n = C + 1; }
				}
				if (n > worst) worst = n;
			}
			if (bad) {
				mism++;
				if (worst > C) casc++;
				else { sumr += worst; hist[worst < 63 ? worst : 63]++; if (worst > maxr) maxr = worst; }
			}
		}
		printf("ch=%d mix=%c C=%ld W=%ld: chunks %ld mismatched %ld (%.3f%%) cascades %ld "
		    "repair mean %.2f max %ld blocks\n", ch, mix, C, W, nch, mism,
		    100.0 * mism / nch, casc, mism - casc ? sumr / (mism - casc) : 0.0, maxr);
	}
	return 0;
}
