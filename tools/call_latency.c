/*
 * call_latency.c -- per-call cost of the host API by call size, CPU core
 * against GPU: bjxa_decode()/bjxa_encode() with n effective blocks per
 * call on 8-bit stereo, 8-bit mono and 4-bit mono (the reference CLI's
 * default incremental shape is n = 1, src/bjxa_decode.c:102-155).  The
 * crossover sizes set the default offload thresholds (libbjxa.c,
 * DESIGN.md §1 "Routing").  Measured in C so the numbers are the
 * library's, not a binding's.
 *
 * build: gcc -O2 -I include -o /tmp/call_latency tools/call_latency.c \
 *            bjxa_amd/libbjxa.so.0 -Wl,-rpath,$PWD/bjxa_amd
 * usage: call_latency [--quick]     (prints one JSON object)
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <time.h>

#include "bjxa.h"
#include "bjxa_hip.h"

static double
now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static uint64_t rng = 0x9e3779b97f4a7c15ull;

static uint8_t
rnd8(void)
{
	rng ^= rng << 13;
	rng ^= rng >> 7;
	rng ^= rng << 17;
	return (uint8_t)(rng >> 24);
}

static void
route(int64_t thr)
{
	(void)bjxa_hip_offload_threshold(BJXA_HIP_OFFLOAD_DECODE, thr);
	(void)bjxa_hip_offload_threshold(BJXA_HIP_OFFLOAD_ENCODE, thr);
}

/* seconds per call of n eblocks */
static double
decode_call(uint32_t n, unsigned bits, unsigned ch)
{
	const uint32_t calls = n >= 200000 ? 5 : (400000 / n < 5 ? 5 :
	    400000 / n > 4000 ? 4000 : 400000 / n);
	const size_t bx = (bits * 4 + 1) * ch, eb = (size_t)n * calls;
	uint8_t *xa = malloc(eb * bx), *pcm = malloc((size_t)n * 64 * ch);
	uint8_t hdr[32] = "KWD1";
	bjxa_decoder_t *d = bjxa_decoder();
	uint32_t v;
	double t;

	for (size_t i = 0; i < eb * bx; i++)
		xa[i] = rnd8();
	for (size_t i = 0; i < eb * ch; i++)	/* gains 0-4 */
		xa[i * (bits * 4 + 1)] = (uint8_t)((rnd8() % 5) << 4 | rnd8() % 13);
	v = (uint32_t)(eb * bx);
	memcpy(hdr + 4, &v, 4);
	v = (uint32_t)(eb * 32);
	memcpy(hdr + 8, &v, 4);
	hdr[12] = 0x44;
	hdr[13] = 0xac;
	hdr[14] = (uint8_t)bits;
	hdr[15] = (uint8_t)ch;
	if (bjxa_parse_header(d, hdr, 32) != 32) {
		perror("bjxa_parse_header");
		exit(1);
	}
	if (bjxa_decode(d, pcm, (size_t)n * 64 * ch, xa, n * bx) != (int)n) {
		perror("bjxa_decode");
		exit(1);
	}
	t = now();
	for (uint32_t c = 1; c < calls; c++)
		if (bjxa_decode(d, pcm, (size_t)n * 64 * ch, xa + c * n * bx,
		    n * bx) != (int)n) {
			perror("bjxa_decode");
			exit(1);
		}
	t = (now() - t) / (calls - 1);
	bjxa_free_decoder(&d);
	free(xa);
	free(pcm);
	return t;
}

static double
encode_call(uint32_t n, unsigned bits, unsigned ch)
{
	const uint32_t calls = n >= 200000 ? 5 : (400000 / n < 5 ? 5 :
	    400000 / n > 4000 ? 4000 : 400000 / n);
	const size_t bp = 64 * ch, bx = (bits * 4 + 1) * ch;
	const size_t bytes = (size_t)n * calls * bp;
	uint8_t *pcm = malloc(bytes), *xa = malloc((size_t)n * bx);
	bjxa_encoder_t *e = bjxa_encoder();
	bjxa_format_t f;
	double t;

	for (size_t i = 0; i < bytes; i++)
		pcm[i] = rnd8();
	memset(&f, 0, sizeof f);
	f.data_len_pcm = (uint32_t)bytes;
	f.samples_rate = 44100;
	f.sample_bits = 16;
	f.channels = (uint8_t)ch;
	if (bjxa_encode_init(e, &f, (uint8_t)bits) < 0 ||
	    bjxa_encode(e, xa, n * bx, pcm, n * bp) != (int)n) {
		perror("bjxa_encode");
		exit(1);
	}
	t = now();
	for (uint32_t c = 1; c < calls; c++)
		if (bjxa_encode(e, xa, n * bx, pcm + c * n * bp, n * bp) !=
		    (int)n) {
			perror("bjxa_encode");
			exit(1);
		}
	t = (now() - t) / (calls - 1);
	bjxa_free_encoder(&e);
	free(pcm);
	free(xa);
	return t;
}

int
main(int argc, char **argv)
{
	static const uint32_t sizes[] = { 1, 4, 16, 64, 256, 512, 1024, 2048,
	    4096, 8192, 16384, 65536, 262144 };
	static const unsigned fmts[][2] = { { 8, 2 }, { 8, 1 }, { 4, 1 } };
	const int quick = argc > 1 && strcmp(argv[1], "--quick") == 0;
	const char *sep = "";

	printf("{");
	for (int dir = 0; dir < 2; dir++) {
		printf("%s\"%s\": {", dir ? ", " : "", dir ? "encode" : "decode");
		for (int f = 0; f < 3; f++) {
			printf("%s\"%u-bit %s\": {", f ? ", " : "", fmts[f][0],
			    fmts[f][1] == 2 ? "stereo" : "mono");
			sep = "";
			for (size_t k = 0; k < sizeof sizes / sizeof *sizes;
			    k += quick ? 2 : 1) {
				const uint32_t n = sizes[k];
				double tc, tg;
				route(INT64_MAX);
				tc = dir ? encode_call(n, fmts[f][0], fmts[f][1]) :
				    decode_call(n, fmts[f][0], fmts[f][1]);
				route(0);
				tg = dir ? encode_call(n, fmts[f][0], fmts[f][1]) :
				    decode_call(n, fmts[f][0], fmts[f][1]);
				printf("%s\"%u\": {\"cpu_us\": %.3f, \"gpu_us\": "
				    "%.3f, \"cpu_MSps\": %.1f, \"gpu_MSps\": %.1f}",
				    sep, n, tc * 1e6, tg * 1e6,
				    n * 32.0 * fmts[f][1] / tc / 1e6,
				    n * 32.0 * fmts[f][1] / tg / 1e6);
				fflush(stdout);
				sep = ", ";
			}
			printf("}");
		}
		printf("}");
	}
	printf("}\n");
	return 0;
}
