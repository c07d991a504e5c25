/*
 * test_api.c -- errno/ownership contract of the C API, case for case the
 * checks of the reference's test/test_libbjxa_api.c:40-296, run against
 * the MI355X libbjxa.so.0.
 *
 * usage: test_api <golden-dir> [<wav-out>]
 *   Every case runs the same with or without a GPU: small calls go to the
 *   library's CPU core, and without a GPU every call does (the test that
 *   runs this under -m gpu sets BJXA_OFFLOAD_DECODE/ENCODE=0 to send the
 *   same calls to the kernels).  With <wav-out>, the mono 4-bit fixture is
 *   also decoded one block per call -- the reference CLI's default loop,
 *   src/bjxa_decode.c:102-155 -- into that WAV file, whose SHA-1 the caller
 *   checks against test/test_decode.sh's.
 */
#ifdef NDEBUG
#undef NDEBUG
#endif
#define _POSIX_C_SOURCE 200809L

#include <assert.h>
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <zlib.h>

#include "bjxa.h"

static const char junk_text[] = "random junk";
static char src_buf[4096];
static char dst_buf[4096];
static const char *golden;

/* the mono 4-bit fixture's header (the reference opens test/square-mono-4.xa) */
static FILE *
open_fixture(void)
{
	char path[4096];
	static unsigned char buf[1 << 20];
	gzFile gz;
	int n;
	FILE *f;

	snprintf(path, sizeof path, "%s/square-mono-4.xa.gz", golden);
	gz = gzopen(path, "rb");
	assert(gz != NULL);
	n = gzread(gz, buf, sizeof buf);
	assert(n > 32);
	gzclose(gz);
	f = fmemopen(buf, (size_t)n, "r");
	assert(f != NULL);
	return (f);
}

static void
check_memory_management(void)
{
	bjxa_decoder_t *dec = bjxa_decoder();
	void *junk = strdup(junk_text);

	assert(dec != NULL && junk != NULL);
	assert(bjxa_free_decoder(NULL) == -1 && errno == EFAULT);
	assert(bjxa_free_decoder(&dec) == 0 && dec == NULL);
	assert(bjxa_free_decoder(&dec) == -1 && errno == EFAULT);
	dec = junk;
	assert(bjxa_free_decoder(&dec) == -1 && errno == EINVAL);
	assert(dec != NULL);
	free(junk);

	bjxa_encoder_t *enc = bjxa_encoder();
	assert(enc != NULL);
	assert(bjxa_free_encoder(NULL) == -1 && errno == EFAULT);
	assert(bjxa_free_encoder(&enc) == 0 && enc == NULL);
	assert(bjxa_free_encoder(&enc) == -1 && errno == EFAULT);
}

static void
check_header_parsing(void)
{
	bjxa_decoder_t *dec = bjxa_decoder();
	void *junk = strdup(junk_text);

	assert(bjxa_parse_header(NULL, junk, 32) == -1 && errno == EFAULT);
	assert(bjxa_parse_header(junk, junk, 32) == -1 && errno == EINVAL);
	assert(bjxa_parse_header(dec, NULL, 32) == -1 && errno == EFAULT);
	assert(bjxa_parse_header(dec, junk, 0) == -1 && errno == ENOBUFS);
	assert(bjxa_fread_header(NULL, stdin) == -1 && errno == EFAULT);
	assert(bjxa_fread_header(junk, stdin) == -1 && errno == EINVAL);
	assert(bjxa_fread_header(dec, NULL) == -1 && errno == EFAULT);
	assert(bjxa_free_decoder(&dec) == 0);
	free(junk);
}

static void
check_file_format(void)
{
	bjxa_decoder_t *dec = bjxa_decoder();
	bjxa_format_t fmt;
	void *junk = strdup(junk_text);

	assert(bjxa_decode_format(NULL, &fmt) == -1 && errno == EFAULT);
	assert(bjxa_decode_format(junk, &fmt) == -1 && errno == EINVAL);
	assert(bjxa_decode_format(dec, &fmt) == -1 && errno == EINVAL);
	assert(bjxa_decode_format(dec, NULL) == -1 && errno == EFAULT);
	assert(bjxa_free_decoder(&dec) == 0);
	free(junk);
}

static void
check_decoding(void)
{
	bjxa_decoder_t *dec = bjxa_decoder();
	bjxa_format_t fmt;
	void *junk = strdup(junk_text);
	FILE *file;

	assert(bjxa_decode(NULL, dst_buf, sizeof dst_buf, src_buf,
	    sizeof src_buf) == -1 && errno == EFAULT);
	assert(bjxa_decode(junk, dst_buf, sizeof dst_buf, src_buf,
	    sizeof src_buf) == -1 && errno == EINVAL);
	assert(bjxa_decode(dec, dst_buf, sizeof dst_buf, src_buf,
	    sizeof src_buf) == -1 && errno == EINVAL);

	file = open_fixture();
	assert(bjxa_fread_header(dec, file) > 0);
	assert(bjxa_decode(dec, NULL, sizeof dst_buf, src_buf,
	    sizeof src_buf) == -1 && errno == EFAULT);
	assert(bjxa_decode(dec, dst_buf, 0, src_buf, sizeof src_buf) == -1 &&
	    errno == ENOBUFS);
	assert(bjxa_decode(dec, dst_buf, sizeof dst_buf, NULL,
	    sizeof src_buf) == -1 && errno == EFAULT);
	assert(bjxa_decode(dec, dst_buf, sizeof dst_buf, src_buf, 0) == -1 &&
	    errno == ENOBUFS);
	assert(bjxa_decode_format(dec, &fmt) == 0);

	/* dst room for 2 blocks, src for 1 -> 1; and the converse */
	memset(src_buf, 0, sizeof src_buf);
	assert(bjxa_decode(dec, dst_buf, fmt.block_size_pcm * 2,
	    src_buf, fmt.block_size_xa) == 1);
	assert(bjxa_decode(dec, dst_buf, fmt.block_size_pcm,
	    src_buf, fmt.block_size_xa * 2) == 1);
	/* past the last block */
	while (bjxa_decode(dec, dst_buf, fmt.block_size_pcm, src_buf,
	    fmt.block_size_xa) == 1)
		;
	assert(errno == EPROTO);
	assert(bjxa_free_decoder(&dec) == 0);
	free(junk);
	fclose(file);
}

static void
check_riff_header_dumping(void)
{
	bjxa_decoder_t *dec = bjxa_decoder();
	void *junk = strdup(junk_text);
	FILE *file;

	assert(bjxa_fwrite_riff_header(NULL, stdout) == -1 && errno == EFAULT);
	assert(bjxa_fwrite_riff_header(junk, stdout) == -1 && errno == EINVAL);
	assert(bjxa_fwrite_riff_header(dec, stdout) == -1 && errno == EINVAL);
	assert(bjxa_dump_riff_header(NULL, dst_buf, sizeof dst_buf) == -1 &&
	    errno == EFAULT);
	assert(bjxa_dump_riff_header(junk, dst_buf, sizeof dst_buf) == -1 &&
	    errno == EINVAL);
	assert(bjxa_dump_riff_header(dec, dst_buf, sizeof dst_buf) == -1 &&
	    errno == EINVAL);

	file = open_fixture();
	assert(bjxa_fread_header(dec, file) > 0);
	assert(bjxa_fwrite_riff_header(dec, NULL) == -1 && errno == EFAULT);
	assert(bjxa_fwrite_riff_header(dec, stdin) == -1 && errno == EBADF);
	assert(bjxa_dump_riff_header(dec, NULL, sizeof dst_buf) == -1 &&
	    errno == EFAULT);
	assert(bjxa_dump_riff_header(dec, dst_buf, 0) == -1 && errno == ENOBUFS);
	assert(bjxa_dump_riff_header(dec, dst_buf, sizeof dst_buf) == 44);
	assert(memcmp(dst_buf, "RIFF", 4) == 0);
	assert(bjxa_free_decoder(&dec) == 0);
	free(junk);
	fclose(file);
}

static void
check_pcm_samples_dumping(void)
{
	const void *src = src_buf;
	void *dst = dst_buf;

	assert(bjxa_dump_pcm(NULL, src, 32) == -1 && errno == EFAULT);
	assert(bjxa_dump_pcm(dst, NULL, 32) == -1 && errno == EFAULT);
	assert(bjxa_dump_pcm(dst, src, 0) == -1 && errno == ENOBUFS);
	assert(bjxa_dump_pcm(dst, src, 31) == -1 && errno == ENOBUFS);
	assert(bjxa_fwrite_pcm(NULL, 32, stdout) == -1 && errno == EFAULT);
	assert(bjxa_fwrite_pcm(src, 0, stdout) == -1 && errno == ENOBUFS);
	assert(bjxa_fwrite_pcm(src, 31, stdout) == -1 && errno == ENOBUFS);
	assert(bjxa_fwrite_pcm(src, 32, NULL) == -1 && errno == EFAULT);
	assert(bjxa_fwrite_pcm(src, 32, stdin) == -1 && errno == EBADF);
}

static void
check_encoder(void)
{
	bjxa_encoder_t *enc = bjxa_encoder();
	bjxa_format_t fmt, out;
	char hdr[64];
	void *junk = strdup(junk_text);

	memset(&fmt, 0, sizeof fmt);
	assert(bjxa_encode_init(NULL, &fmt, 8) == -1 && errno == EFAULT);
	assert(bjxa_encode_init(junk, &fmt, 8) == -1 && errno == EINVAL);
	assert(bjxa_encode_init(enc, NULL, 8) == -1 && errno == EFAULT);
	assert(bjxa_encode_init(enc, &fmt, 8) == -1 && errno == EINVAL);
	fmt.sample_bits = 16;
	assert(bjxa_encode_init(enc, &fmt, 5) == -1 && errno == EINVAL);
	assert(bjxa_encode_init(enc, &fmt, 8) == -1 && errno == EPROTO);
	assert(bjxa_encode_format(enc, &out) == -1 && errno == EINVAL);
	assert(bjxa_dump_header(enc, hdr, sizeof hdr) == -1 && errno == EINVAL);
	assert(bjxa_encode(enc, dst_buf, sizeof dst_buf, src_buf,
	    sizeof src_buf) == -1 && errno == EINVAL);

	fmt.channels = 2;
	fmt.samples_rate = 44100;
	fmt.data_len_pcm = 4 * 100;		/* 100 frames */
	assert(bjxa_encode_init(enc, &fmt, 6) == 0);
	assert(fmt.blocks == 4 && fmt.block_size_xa == 50 &&
	    fmt.block_size_pcm == 128);
	assert(bjxa_encode_format(enc, &out) == 0);
	assert(out.sample_bits == 6 && out.blocks == 4 && out.data_len_pcm == 400);
	assert(bjxa_dump_header(enc, hdr, 31) == -1 && errno == ENOBUFS);
	assert(bjxa_dump_header(enc, hdr, sizeof hdr) == 32);
	assert(memcmp(hdr, "KWD1", 4) == 0 && (unsigned char)hdr[4] == 200 &&
	    hdr[14] == 6 && hdr[15] == 2);
	assert(bjxa_encode(enc, dst_buf, 49, src_buf, sizeof src_buf) == -1 &&
	    errno == ENOBUFS);
	assert(bjxa_encode(enc, dst_buf, 50, src_buf, 127) == -1 &&
	    errno == ENOBUFS);
	assert(bjxa_encode(enc, dst_buf, 200, src_buf, 400) == 4);
	assert(bjxa_free_encoder(&enc) == 0);
	free(junk);
}

/* the fixture through one bjxa_decode() per block into a WAV file */
static void
decode_fixture(const char *path)
{
	bjxa_decoder_t *dec = bjxa_decoder();
	bjxa_format_t fmt;
	FILE *in = open_fixture(), *out = fopen(path, "wb");
	uint32_t left;

	assert(dec != NULL && out != NULL);
	assert(bjxa_fread_header(dec, in) == 32);
	assert(bjxa_decode_format(dec, &fmt) == 0);
	assert(bjxa_fwrite_riff_header(dec, out) == 44);
	left = fmt.data_len_pcm;
	while (fmt.blocks-- > 0) {
		const uint32_t n = left < fmt.block_size_pcm ? left :
		    fmt.block_size_pcm;
		assert(fread(src_buf, fmt.block_size_xa, 1, in) == 1);
		assert(bjxa_decode(dec, dst_buf, fmt.block_size_pcm, src_buf,
		    fmt.block_size_xa) == 1);
		assert(bjxa_fwrite_pcm((int16_t *)(void *)dst_buf, n, out) == 0);
		left -= n;
	}
	assert(left == 0);
	assert(bjxa_decode(dec, dst_buf, fmt.block_size_pcm, src_buf,
	    fmt.block_size_xa) == -1 && errno == EPROTO);
	assert(bjxa_free_decoder(&dec) == 0);
	fclose(in);
	assert(fclose(out) == 0);
}

int
main(int argc, char **argv)
{
	assert(argc >= 2);
	golden = argv[1];
	assert(sizeof(bjxa_format_t) == 16);
	check_memory_management();
	check_header_parsing();
	check_file_format();
	check_decoding();
	check_riff_header_dumping();
	check_pcm_samples_dumping();
	check_encoder();
	if (argc > 2)
		decode_fixture(argv[2]);
	puts("test_api: ok");
	return (EXIT_SUCCESS);
}
