/*
 * bjxa_cli.c -- the bjxa(1) command over libbjxa.so.0 (MI355X build).
 *
 * Command line, messages and exit status follow the reference CLI
 * (src/bjxa.c:34-145, src/bjxa_decode.c, src/bjxa_encode.c), whose tests
 * (test/test_bjxa.sh, test/test_decode.sh, test/test_decode_error.sh) are
 * re-run against this binary by tests/test_cli.py:
 *
 *   bjxa help
 *   bjxa decode [<xa file> [<wav file>]]
 *   bjxa encode [--bits <4|6|8>] [<wav file> [<xa file>]]
 *
 * A missing file operand or "-" is standard input/output.  Failures print
 * "bjxa: <reason>" plus the usage for command-line errors, "Error: ..." for
 * files that cannot be opened, and "<libbjxa call>: <strerror>" for codec
 * errors; the exit status is then 1.
 *
 * Call shape: one bjxa_decode()/bjxa_encode() per stream -- the reference's
 * BJXA_SINGLE_PASS build (src/bjxa_decode.c:56-100, src/bjxa_encode.c:
 * 62-110) and the shape the GPU path is built for.  BJXA_CLI_BLOCKS=1 in
 * the environment selects the reference's default one-block-per-call loop
 * (src/bjxa_decode.c:102-155) instead; the output is the same.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "bjxa.h"		/* expects <stdio.h> and ssize_t, as the reference's */

static const char *prog = "bjxa";

static void
usage(FILE *f)
{
	fprintf(f,
	    "Usage: %s <action> [args...]\n"
	    "\n"
	    "Actions:\n"
	    "\n"
	    "  help\n"
	    "    Print this text.\n"
	    "\n"
	    "  decode [<xa file> [<wav file>]]\n"
	    "    Convert an XA file into a WAV file.\n"
	    "\n"
	    "  encode [--bits <4|6|8>] [<wav file> [<xa file>]]\n"
	    "    Convert a WAV file into an XA file, with 6 bits per sample\n"
	    "    unless --bits says otherwise.\n"
	    "\n"
	    "A missing file name, or \"-\", means standard input or output.\n",
	    prog);
}

static void
bad_usage(const char *reason)
{
	fprintf(stderr, "bjxa: %s\n", reason);
	usage(stderr);
	exit(EXIT_FAILURE);
}

/* point stdin/stdout at the file operands */
static int
redirect(int argc, char *const *argv)
{
	if (argc > 0 && strcmp(argv[0], "-") != 0 &&
	    freopen(argv[0], "rb", stdin) == NULL) {
		perror("Error");
		return (-1);
	}
	if (argc > 1 && strcmp(argv[1], "-") != 0 &&
	    freopen(argv[1], "wb", stdout) == NULL) {
		perror("Error");
		return (-1);
	}
	return (0);
}

static int
read_exact(void *buf, size_t len, FILE *in)
{
	if (len == 0 || fread(buf, len, 1, in) == 1)
		return (0);
	if (feof(in))
		fprintf(stderr, "fread: End of file\n");
	else
		perror("fread");
	return (-1);
}

static int
block_calls(void)
{
	const char *e = getenv("BJXA_CLI_BLOCKS");
	return (e != NULL && *e != '\0' && strcmp(e, "0") != 0);
}

/* one call over the whole stream */
static int
decode_stream(bjxa_decoder_t *dec, const bjxa_format_t *fmt, FILE *in,
    FILE *out)
{
	const size_t xa_len = (size_t)fmt->block_size_xa * fmt->blocks;
	void *xa = malloc(xa_len + 1), *pcm = malloc((size_t)fmt->data_len_pcm + 1);
	int rc = -1;

	if (xa == NULL || pcm == NULL)
		perror("malloc");
	else if (read_exact(xa, xa_len, in) == 0) {
		if (bjxa_decode(dec, pcm, fmt->data_len_pcm, xa, xa_len) !=
		    (int)fmt->blocks)
			perror("bjxa_decode");
		else if (bjxa_fwrite_pcm(pcm, fmt->data_len_pcm, out) < 0)
			perror("bjxa_fwrite_pcm");
		else
			rc = 0;
	}
	free(xa);
	free(pcm);
	return (rc);
}

/* one call per effective block */
static int
decode_blocks(bjxa_decoder_t *dec, const bjxa_format_t *fmt, FILE *in,
    FILE *out)
{
	void *xa = malloc(fmt->block_size_xa), *pcm = malloc(fmt->block_size_pcm);
	uint32_t left = fmt->data_len_pcm;
	int rc = 0;

	if (xa == NULL || pcm == NULL) {
		perror("malloc");
		rc = -1;
	}
	for (uint32_t b = 0; rc == 0 && b < fmt->blocks; b++) {
		const uint32_t n = left < fmt->block_size_pcm ? left :
		    fmt->block_size_pcm;
		if (read_exact(xa, fmt->block_size_xa, in) < 0)
			rc = -1;
		else if (bjxa_decode(dec, pcm, fmt->block_size_pcm, xa,
		    fmt->block_size_xa) != 1) {
			perror("bjxa_decode");
			rc = -1;
		} else if (bjxa_fwrite_pcm(pcm, n, out) < 0) {
			perror("bjxa_fwrite_pcm");
			rc = -1;
		}
		left -= n;
	}
	free(xa);
	free(pcm);
	return (rc);
}

static int
cmd_decode(FILE *in, FILE *out)
{
	bjxa_decoder_t *dec = bjxa_decoder();
	bjxa_format_t fmt;
	int rc = -1;

	if (dec == NULL) {
		perror("bjxa_decoder");
		return (-1);
	}
	if (bjxa_fread_header(dec, in) < 0)
		perror("bjxa_fread_header");
	else if (bjxa_decode_format(dec, &fmt) < 0)
		perror("bjxa_decode_format");
	else if (bjxa_fwrite_riff_header(dec, out) < 0)
		perror("bjxa_fwrite_riff_header");
	else
		rc = block_calls() ? decode_blocks(dec, &fmt, in, out) :
		    decode_stream(dec, &fmt, in, out);
	if (bjxa_free_decoder(&dec) < 0) {
		perror("bjxa_free_decoder");
		rc = -1;
	}
	return (rc);
}

static int
encode_stream(bjxa_encoder_t *enc, const bjxa_format_t *fmt, FILE *in,
    FILE *out)
{
	const size_t xa_len = (size_t)fmt->block_size_xa * fmt->blocks;
	void *xa = malloc(xa_len + 1), *pcm = malloc((size_t)fmt->data_len_pcm + 1);
	int rc = -1;

	if (xa == NULL || pcm == NULL)
		perror("malloc");
	else if (read_exact(pcm, fmt->data_len_pcm, in) == 0) {
		if (bjxa_encode(enc, xa, xa_len, pcm, fmt->data_len_pcm) !=
		    (int)fmt->blocks)
			perror("bjxa_encode");
		else if (xa_len > 0 && fwrite(xa, xa_len, 1, out) != 1)
			perror("fwrite");
		else
			rc = 0;
	}
	free(xa);
	free(pcm);
	return (rc);
}

static int
encode_blocks(bjxa_encoder_t *enc, const bjxa_format_t *fmt, FILE *in,
    FILE *out)
{
	void *xa = malloc(fmt->block_size_xa), *pcm = malloc(fmt->block_size_pcm);
	uint32_t left = fmt->data_len_pcm;
	int rc = 0;

	if (xa == NULL || pcm == NULL) {
		perror("malloc");
		rc = -1;
	}
	for (uint32_t b = 0; rc == 0 && b < fmt->blocks; b++) {
		const uint32_t n = left < fmt->block_size_pcm ? left :
		    fmt->block_size_pcm;
		if (read_exact(pcm, n, in) < 0)
			rc = -1;
		else if (bjxa_encode(enc, xa, fmt->block_size_xa, pcm,
		    fmt->block_size_pcm) != 1) {
			perror("bjxa_encode");
			rc = -1;
		} else if (fwrite(xa, fmt->block_size_xa, 1, out) != 1) {
			perror("fwrite");
			rc = -1;
		}
		left -= n;
	}
	free(xa);
	free(pcm);
	return (rc);
}

static int
cmd_encode(FILE *in, FILE *out, unsigned bits)
{
	bjxa_encoder_t *enc = bjxa_encoder();
	bjxa_format_t fmt;
	int rc = -1;

	if (enc == NULL) {
		perror("bjxa_encoder");
		return (-1);
	}
	if (bjxa_fread_riff_header(&fmt, in) < 0)
		perror("bjxa_fread_riff_header");
	else if (bjxa_encode_init(enc, &fmt, (uint8_t)bits) < 0)
		perror("bjxa_encode_init");
	else if (bjxa_encode_format(enc, &fmt) < 0)
		perror("bjxa_encode_format");
	else if (bjxa_fwrite_header(enc, out) < 0)
		perror("bjxa_fwrite_header");
	else
		rc = block_calls() ? encode_blocks(enc, &fmt, in, out) :
		    encode_stream(enc, &fmt, in, out);
	if (bjxa_free_encoder(&enc) < 0) {
		perror("bjxa_free_encoder");
		rc = -1;
	}
	return (rc);
}

int
main(int argc, char **argv)
{
	if (argc > 0)
		prog = argv[0];
	if (argc < 2)
		bad_usage("Missing an action");
	const char *action = argv[1];
	argc -= 2;
	argv += 2;

	if (strcmp(action, "help") == 0) {
		usage(stdout);
		return (EXIT_SUCCESS);
	}
	if (strcmp(action, "decode") == 0) {
		if (argc > 2)
			bad_usage("Too many arguments");
		if (redirect(argc, argv) < 0 || cmd_decode(stdin, stdout) < 0)
			return (EXIT_FAILURE);
		return (EXIT_SUCCESS);
	}
	if (strcmp(action, "encode") == 0) {
		unsigned bits = 6;
		if (argc > 0 && strcmp(argv[0], "--bits") == 0) {
			if (argc < 2)
				bad_usage("Missing number of bits per sample");
			const char *v = argv[1];
			if (strcmp(v, "4") != 0 && strcmp(v, "6") != 0 &&
			    strcmp(v, "8") != 0)
				bad_usage("Invalid number of bits per sample");
			bits = (unsigned)(v[0] - '0');
			argc -= 2;
			argv += 2;
		}
		if (argc > 2)
			bad_usage("Too many arguments");
		if (redirect(argc, argv) < 0 || cmd_encode(stdin, stdout, bits) < 0)
			return (EXIT_FAILURE);
		return (EXIT_SUCCESS);
	}
	bad_usage("Unknown action");
	return (EXIT_FAILURE);
}
