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
 * Call shape: by default the whole stream is read and handed to one
 * bjxa_decode()/bjxa_encode() call -- the reference's BJXA_SINGLE_PASS shape
 * (src/bjxa_decode.c:56-100, src/bjxa_encode.c:62-110), which lets a large
 * stream run on the GPU -- but the output on failure is that of the
 * reference's default one-block-per-call loop (src/bjxa_decode.c:102-155,
 * src/bjxa_encode.c:108-176): a stream cut short yields every whole block
 * that was read, then "fread: End of file"; a block whose gain nibble is
 * >= 5 yields the PCM of every block before it, then "bjxa_decode:
 * Protocol error".  BJXA_CLI_BLOCKS=1 selects the one-block-per-call loop
 * itself; both shapes write the same bytes.
 */
#include <errno.h>
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

static void
read_error(FILE *in)
{
	if (feof(in))
		fprintf(stderr, "fread: End of file\n");
	else
		perror("fread");
}

static int
read_exact(void *buf, size_t len, FILE *in)
{
	if (len == 0 || fread(buf, len, 1, in) == 1)
		return (0);
	read_error(in);
	return (-1);
}

/* first eblock of `n` holding a channel block whose gain nibble is >= 5
 * (the reference's EPROTO, src/libbjxa.c:547-550), or n */
static uint32_t
first_bad_block(const uint8_t *xa, uint32_t n, const bjxa_format_t *fmt)
{
	const unsigned bsz = fmt->block_size_xa / fmt->channels;
	for (uint32_t b = 0; b < n; b++)
		for (unsigned c = 0; c < fmt->channels; c++)
			if (xa[(size_t)b * fmt->block_size_xa + c * bsz] >= 0x50)
				return (b);
	return (n);
}

static int
block_calls(void)
{
	const char *e = getenv("BJXA_CLI_BLOCKS");
	return (e != NULL && *e != '\0' && strcmp(e, "0") != 0);
}

/*
 * One call over the whole stream, with the per-block loop's output on
 * failure: the PCM of the whole blocks that were read (up to a bad block)
 * is written before the error is reported.
 */
static int
decode_stream(bjxa_decoder_t *dec, const bjxa_format_t *fmt, FILE *in,
    FILE *out)
{
	/* room for one whole block even when the stream is shorter, as the
	 * per-block loop passes (a sub-block single pass is ENOBUFS) */
	const size_t pcm_len = fmt->data_len_pcm > fmt->block_size_pcm ?
	    fmt->data_len_pcm : fmt->block_size_pcm;
	uint8_t *xa = malloc((size_t)fmt->block_size_xa * fmt->blocks + 1);
	void *pcm = malloc(pcm_len);
	uint32_t got, good;
	size_t bytes;
	int rc = -1, bad = 0;

	if (xa == NULL || pcm == NULL) {
		perror("malloc");
		goto done;
	}
	got = (uint32_t)fread(xa, fmt->block_size_xa, fmt->blocks, in);
	good = got;
	if (got > 0 && bjxa_decode(dec, pcm, pcm_len, xa,
	    (size_t)got * fmt->block_size_xa) != (int)got) {
		const int e = errno;
		/* only a bad profile (EPROTO) leaves the PCM before it in the
		 * buffer; any other failure (EIO, ENOMEM, ENODEV from the
		 * device path) decoded nothing there, so nothing is written */
		good = e == EPROTO ? first_bad_block(xa, got, fmt) : 0;
		bad = 1;
		errno = e;
	}
	bytes = (size_t)good * fmt->block_size_pcm;
	if (bytes > fmt->data_len_pcm)
		bytes = fmt->data_len_pcm;
	if (bad) {
		const int e = errno;
		if (bytes > 0)
			(void)bjxa_fwrite_pcm(pcm, bytes, out);
		errno = e;
		perror("bjxa_decode");
	} else if (bytes > 0 && bjxa_fwrite_pcm(pcm, bytes, out) < 0) {
		perror("bjxa_fwrite_pcm");
	} else if (got < fmt->blocks) {
		read_error(in);
	} else {
		rc = 0;
	}
done:
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

/* one call over the whole stream; on a short read, the XA of the blocks
 * whose PCM was complete is written before the error (as the per-block
 * loop does) */
static int
encode_stream(bjxa_encoder_t *enc, const bjxa_format_t *fmt, FILE *in,
    FILE *out)
{
	const size_t xa_len = (size_t)fmt->block_size_xa * fmt->blocks;
	const size_t pcm_len = fmt->data_len_pcm > fmt->block_size_pcm ?
	    fmt->data_len_pcm : fmt->block_size_pcm;
	void *xa = malloc(xa_len + 1), *pcm = malloc(pcm_len);
	size_t got;
	uint32_t n;
	int rc = -1;

	if (xa == NULL || pcm == NULL) {
		perror("malloc");
		goto done;
	}
	got = fread(pcm, 1, fmt->data_len_pcm, in);
	n = got == fmt->data_len_pcm ? fmt->blocks :
	    (uint32_t)(got / fmt->block_size_pcm);
	if (n > 0 && bjxa_encode(enc, xa, xa_len, pcm, got == fmt->data_len_pcm ?
	    pcm_len : (size_t)n * fmt->block_size_pcm) != (int)n)
		perror("bjxa_encode");
	else if (n > 0 && fwrite(xa, (size_t)n * fmt->block_size_xa, 1, out) != 1)
		perror("fwrite");
	else if (n < fmt->blocks)
		read_error(in);
	else
		rc = 0;
done:
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
