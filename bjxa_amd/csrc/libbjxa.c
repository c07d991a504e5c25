/*
 * libbjxa.c -- host side of the MI355X libbjxa: codec objects, XA header
 * and RIFF/WAVE framing, the errno contract, and per-call bookkeeping.
 * The block arithmetic of bjxa_decode()/bjxa_encode() runs on the GPU
 * (xa_decode.hip / xa_encode.hip via xa_gpu.hip) for calls of at least
 * the offload threshold, and on the calling thread's core (xa_cpu.c) for
 * smaller calls and on hosts without a GPU ("Routing").
 *
 * Each entry point restates the behaviour of the reference routine cited
 * next to it (paths relative to the reference checkout), including its
 * argument-check order, errno values and the 32-bit arithmetic quirks of
 * header validation.
 */
#define _POSIX_C_SOURCE 200809L

#include <assert.h>
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "bjxa.h"
#include "bjxa_hip.h"
#include "xa_gpu.h"

#define XA_FRAMES	32
#define DEC_MAGIC	0x6a78ad3cu
#define ENC_MAGIC	0x6a78e5c1u

struct bjxa_decoder {
	uint32_t		magic;
	uint32_t		data_len;	/* XA payload bytes (header) */
	uint32_t		samples;	/* frames (header) */
	uint16_t		rate;
	uint8_t			bits;
	uint8_t			block_size;	/* per channel: bits*4+1 */
	uint8_t			channels;
	int16_t			state[4];	/* L p0, L p1, R p0, R p1 */
	bjxa_format_t		left;		/* remaining work */
	struct bjxa__gpu	*gpu;
};

struct bjxa_encoder {
	uint32_t		magic;
	uint32_t		data_len;	/* XA payload bytes to produce */
	uint32_t		samples;
	uint16_t		rate;
	uint8_t			bits;
	uint8_t			block_size;
	uint8_t			channels;
	bjxa_format_t		left;
	struct bjxa__gpu	*gpu;
};

/* argument checks, in the reference's order (src/libbjxa.c:53-97) */
#define FAIL(err)	do { errno = (err); return (-1); } while (0)
#define NEED_PTR(p)	do { if ((p) == NULL) FAIL(EFAULT); } while (0)
#define NEED_OBJ(o, m)	do { NEED_PTR(o); if ((o)->magic != (m)) \
			    FAIL(EINVAL); } while (0)
#define REQUIRE(c, err)	do { if (!(c)) FAIL(err); } while (0)

/* little-endian field access */
static uint32_t
get_le(const uint8_t *p, unsigned n)
{
	uint32_t v = 0;
	while (n-- > 0)
		v = (v << 8) | p[n];
	return (v);
}

static uint8_t *
put_le(uint8_t *p, uint32_t v, unsigned n)
{
	while (n-- > 0) {
		*p++ = (uint8_t)v;
		v >>= 8;
	}
	return (p);
}

static uint8_t *
put_tag(uint8_t *p, const char *tag)
{
	size_t n = strlen(tag);
	memcpy(p, tag, n);
	return (p + n);
}

/* read exactly n bytes; EIO on a short read at end of file */
static int
read_all(void *buf, size_t n, FILE *file)
{
	if (fread(buf, n, 1, file) != 1) {
		if (feof(file))
			errno = EIO;
		return (-1);
	}
	return (0);
}

/* ---- CPU / GPU routing (LIBBJXA_HIP_0.3) ------------------------------- */

/*
 * A call of at least offload_min[dir] effective blocks runs on the GPU, a
 * smaller one on the calling core.  The unit is the eblock because the CPU
 * core's cost is: a stereo eblock runs its two channel chains side by side
 * in about the time of one mono block.  Defaults are the crossover points
 * measured with tools/call_latency.c on the GPU box (EPYC 9575F host,
 * DESIGN.md §1 "Routing": decode ~1,100 stereo / ~800 mono eblocks, encode
 * ~4,000-5,000); BJXA_OFFLOAD_DECODE and BJXA_OFFLOAD_ENCODE override them
 * at load time, bjxa_hip_offload_threshold() at run time.
 */
#define OFFLOAD_DECODE_DEFAULT	1024u
#define OFFLOAD_ENCODE_DEFAULT	4096u

static uint64_t offload_min[2];
#ifdef BJXA_TEST_HOOKS
static int fault_gpu_decode;	/* BJXA_TEST_FAULT=gpu-decode */
#endif
static pthread_once_t offload_once = PTHREAD_ONCE_INIT;

/* a threshold: decimal digits only, no sign, no blanks, no overflow */
static int
parse_threshold(const char *v, uint64_t *out)
{
	char *end;
	unsigned long long n;

	if (v == NULL || *v < '0' || *v > '9')
		return (-1);
	errno = 0;
	n = strtoull(v, &end, 10);
	if (errno == ERANGE || *end != '\0')
		return (-1);
	*out = (uint64_t)n;
	return (0);
}

static void
offload_init(void)
{
	static const char *const env[2] = { "BJXA_OFFLOAD_DECODE",
	    "BJXA_OFFLOAD_ENCODE" };
	const uint64_t dflt[2] = { OFFLOAD_DECODE_DEFAULT,
	    OFFLOAD_ENCODE_DEFAULT };
	const int saved = errno;

	for (int d = 0; d < 2; d++) {
		const char *v = getenv(env[d]);
		uint64_t n = dflt[d];
		if (v != NULL && *v != '\0' && parse_threshold(v, &n) < 0) {
			fprintf(stderr, "libbjxa: ignoring %s=\"%s\" (not a "
			    "block count); using %llu\n", env[d], v,
			    (unsigned long long)dflt[d]);
			n = dflt[d];
		}
		__atomic_store_n(&offload_min[d], n, __ATOMIC_RELAXED);
	}
#ifdef BJXA_TEST_HOOKS
	/* fault injection for the CLI tests (test build only, make
	 * testhooks): a call routed to the device fails with EIO before
	 * anything is decoded, with or without a GPU */
	{
		const char *f = getenv("BJXA_TEST_FAULT");
		fault_gpu_decode = f != NULL && strcmp(f, "gpu-decode") == 0;
	}
#endif
	errno = saved;
}

static int
on_gpu(int dir, uint64_t eblocks)
{
	(void)pthread_once(&offload_once, offload_init);
	return eblocks >= __atomic_load_n(&offload_min[dir], __ATOMIC_RELAXED) &&
	    bjxa__gpu_present();
}

#ifdef BJXA_TEST_HOOKS
/* BJXA_TEST_FAULT=gpu-decode and a call the threshold sends to the device */
static int
gpu_decode_faulted(uint64_t eblocks)
{
	(void)pthread_once(&offload_once, offload_init);
	return fault_gpu_decode && eblocks >= __atomic_load_n(
	    &offload_min[BJXA_HIP_OFFLOAD_DECODE], __ATOMIC_RELAXED);
}
#endif

int64_t
bjxa_hip_offload_threshold(int direction, int64_t eblocks)
{
	if (direction != BJXA_HIP_OFFLOAD_DECODE &&
	    direction != BJXA_HIP_OFFLOAD_ENCODE) {
		errno = EINVAL;
		return (-1);
	}
	(void)pthread_once(&offload_once, offload_init);
	if (eblocks < 0)
		return ((int64_t)__atomic_load_n(&offload_min[direction],
		    __ATOMIC_RELAXED));
	return ((int64_t)__atomic_exchange_n(&offload_min[direction],
	    (uint64_t)eblocks, __ATOMIC_RELAXED));
}

/* ---- objects (src/libbjxa.c:246-282) --------------------------------- */

bjxa_decoder_t *
bjxa_decoder(void)
{
	bjxa_decoder_t *dec;

	errno = 0;
	dec = calloc(1, sizeof *dec);
	if (dec != NULL)
		dec->magic = DEC_MAGIC;
	return (dec);
}

int
bjxa_free_decoder(bjxa_decoder_t **decp)
{
	bjxa_decoder_t *dec;

	NEED_PTR(decp);
	NEED_OBJ(*decp, DEC_MAGIC);
	dec = *decp;
	*decp = NULL;
	bjxa__gpu_free(dec->gpu);
	memset(dec, 0, sizeof *dec);
	free(dec);
	return (0);
}

bjxa_encoder_t *
bjxa_encoder(void)
{
	bjxa_encoder_t *enc;

	errno = 0;
	enc = calloc(1, sizeof *enc);
	if (enc != NULL)
		enc->magic = ENC_MAGIC;
	return (enc);
}

int
bjxa_free_encoder(bjxa_encoder_t **encp)
{
	bjxa_encoder_t *enc;

	NEED_PTR(encp);
	NEED_OBJ(*encp, ENC_MAGIC);
	enc = *encp;
	*encp = NULL;
	bjxa__gpu_free(enc->gpu);
	memset(enc, 0, sizeof *enc);
	free(enc);
	return (0);
}

/* ---- XA header (src/libbjxa.c:395-521) ------------------------------- */

static void
dec_format(const bjxa_decoder_t *dec, bjxa_format_t *fmt)
{
	/* src/libbjxa.c:588-597: always the whole stream */
	fmt->data_len_pcm = dec->samples * dec->channels * 2u;
	fmt->samples_rate = dec->rate;
	fmt->sample_bits = 16;
	fmt->channels = dec->channels;
	fmt->block_size_xa = (uint8_t)(dec->block_size * dec->channels);
	fmt->block_size_pcm = (uint8_t)(XA_FRAMES * dec->channels * 2u);
	fmt->blocks = dec->data_len / fmt->block_size_xa;
	/* a stereo payload of an odd number of channel blocks passes the
	 * header checks and trips this, as in the reference (:597) */
	assert(fmt->blocks * fmt->block_size_xa == dec->data_len);
}

ssize_t
bjxa_parse_header(bjxa_decoder_t *dec, const void *src, size_t len)
{
	const uint8_t *h = src;
	bjxa_decoder_t tmp;
	uint32_t nblk, max_samples;

	NEED_OBJ(dec, DEC_MAGIC);
	NEED_PTR(src);
	REQUIRE(len >= BJXA_HEADER_SIZE_XA, ENOBUFS);

	memset(&tmp, 0, sizeof tmp);
	REQUIRE(memcmp(h, "KWD1", 4) == 0, EPROTO);
	tmp.data_len = get_le(h + 4, 4);
	tmp.samples = get_le(h + 8, 4);
	tmp.rate = (uint16_t)get_le(h + 12, 2);
	tmp.bits = h[14];
	tmp.channels = h[15];
	/* h[16..19] loop pointer and h[28..31] padding are ignored */
	tmp.state[0] = (int16_t)get_le(h + 20, 2);
	tmp.state[1] = (int16_t)get_le(h + 22, 2);
	tmp.state[2] = (int16_t)get_le(h + 24, 2);
	tmp.state[3] = (int16_t)get_le(h + 26, 2);

	/* validation order and uint32 arithmetic of :425-437 */
	REQUIRE(tmp.data_len > 0, EPROTO);
	REQUIRE(tmp.samples > 0, EPROTO);
	REQUIRE(tmp.rate > 0, EPROTO);
	REQUIRE(tmp.bits == 4 || tmp.bits == 6 || tmp.bits == 8, EPROTO);
	REQUIRE(tmp.channels == 1 || tmp.channels == 2, EPROTO);
	tmp.block_size = (uint8_t)(tmp.bits * 4 + 1);
	nblk = tmp.data_len / tmp.block_size;
	max_samples = (uint32_t)(XA_FRAMES * tmp.data_len) /
	    (uint32_t)(tmp.block_size * tmp.channels);
	REQUIRE(nblk * tmp.block_size == tmp.data_len, EPROTO);
	REQUIRE(max_samples >= tmp.samples, EPROTO);
	REQUIRE(max_samples - tmp.samples < XA_FRAMES, EPROTO);

	dec_format(&tmp, &tmp.left);
	tmp.magic = DEC_MAGIC;
	tmp.gpu = dec->gpu;	/* device buffers survive a re-parse */
	*dec = tmp;
	return (BJXA_HEADER_SIZE_XA);
}

ssize_t
bjxa_fread_header(bjxa_decoder_t *dec, FILE *file)
{
	uint8_t buf[BJXA_HEADER_SIZE_XA];
	ssize_t ret;

	NEED_OBJ(dec, DEC_MAGIC);
	NEED_PTR(file);
	if (read_all(buf, sizeof buf, file) < 0)
		return (-1);
	ret = bjxa_parse_header(dec, buf, sizeof buf);
	assert(ret >= 0 || (errno != EINVAL && errno != ENOBUFS));
	return (ret);
}

ssize_t
bjxa_dump_header(bjxa_encoder_t *enc, void *dst, size_t len)
{
	uint8_t *p = dst;

	NEED_OBJ(enc, ENC_MAGIC);
	NEED_PTR(dst);
	REQUIRE(len >= BJXA_HEADER_SIZE_XA, ENOBUFS);
	REQUIRE(enc->data_len > 0, EINVAL);

	p = put_tag(p, "KWD1");
	p = put_le(p, enc->data_len, 4);
	p = put_le(p, enc->samples, 4);
	p = put_le(p, enc->rate, 2);
	p = put_le(p, enc->bits, 1);
	p = put_le(p, enc->channels, 1);
	memset(p, 0, 16);	/* loop, befL, befR, pad (:495-500) */
	return (BJXA_HEADER_SIZE_XA);
}

ssize_t
bjxa_fwrite_header(bjxa_encoder_t *enc, FILE *file)
{
	uint8_t buf[BJXA_HEADER_SIZE_XA];

	NEED_OBJ(enc, ENC_MAGIC);
	NEED_PTR(file);
	if (bjxa_dump_header(enc, buf, sizeof buf) < 0)
		return (-1);
	if (fwrite(buf, sizeof buf, 1, file) != 1)
		return (-1);
	return (BJXA_HEADER_SIZE_XA);
}

/* ---- decode (src/libbjxa.c:580-661) ---------------------------------- */

int
bjxa_decode_format(bjxa_decoder_t *dec, bjxa_format_t *fmt)
{
	NEED_OBJ(dec, DEC_MAGIC);
	NEED_PTR(fmt);
	REQUIRE(dec->block_size != 0, EINVAL);
	dec_format(dec, fmt);
	return (0);
}

int
bjxa_decode(bjxa_decoder_t *dec, void *dst, size_t dst_len, const void *src,
    size_t src_len)
{
	bjxa_format_t *f;
	uint64_t n, copy;
	uint32_t err_cb;
	int16_t st[4];

	NEED_OBJ(dec, DEC_MAGIC);
	NEED_PTR(dst);
	NEED_PTR(src);
	f = &dec->left;
	REQUIRE(f->sample_bits == 16, EINVAL);
	REQUIRE(f->blocks > 0, EPROTO);
	/* both checks use full block sizes, even for a short last block */
	REQUIRE(dst_len >= f->block_size_pcm, ENOBUFS);
	REQUIRE(src_len >= f->block_size_xa, ENOBUFS);

	/* the reference's per-block loop (:629-658) stops at the first of:
	 * no blocks left, src exhausted, the next block's PCM not fitting */
	n = f->blocks;
	if (src_len / f->block_size_xa < n)
		n = src_len / f->block_size_xa;
	if (dst_len < f->data_len_pcm && dst_len / f->block_size_pcm < n)
		n = dst_len / f->block_size_pcm;
	copy = n * f->block_size_pcm;
	if (copy > f->data_len_pcm)
		copy = f->data_len_pcm;

	memcpy(st, dec->state, sizeof st);
#ifdef BJXA_TEST_HOOKS
	if (gpu_decode_faulted(n))
		FAIL(EIO);
#endif
	if (!on_gpu(BJXA_HIP_OFFLOAD_DECODE, n)) {
		(void)bjxa__cpu_decode(src, (uint32_t)n, dec->bits,
		    dec->channels, st, dst, copy, &err_cb);
	} else {
		if (dec->gpu == NULL && (dec->gpu = bjxa__gpu_new()) == NULL)
			return (-1);
		if (bjxa__gpu_decode(dec->gpu, src, (uint32_t)n, dec->bits,
		    dec->channels, st, dst, copy, &err_cb) < 0)
			return (-1);
	}
	memcpy(dec->state, st, sizeof st);
	if (err_cb != 0xffffffffu) {
		/* gain nibble >= 5 (:550): the eblocks before it are in dst
		 * and accounted for; the call fails with EPROTO */
		uint32_t done = err_cb / dec->channels;
		f->blocks -= done;
		f->data_len_pcm -= done * f->block_size_pcm;
		FAIL(EPROTO);
	}
	f->blocks -= (uint32_t)n;
	f->data_len_pcm -= (uint32_t)copy;
	return ((int)n);
}

/* ---- WAVE (src/libbjxa.c:821-996) ------------------------------------ */

ssize_t
bjxa_parse_riff_header(bjxa_format_t *fmt, const void *src, size_t len)
{
	const uint8_t *h = src;
	uint32_t riff_len, hdr_len, rate, byte_rate, data_len;
	uint16_t tag, chans, align, bits;
	bjxa_format_t out;

	NEED_PTR(fmt);
	NEED_PTR(src);
	REQUIRE(len >= BJXA_HEADER_SIZE_RIFF, ENOBUFS);

	REQUIRE(memcmp(h, "RIFF", 4) == 0, EPROTO);
	riff_len = get_le(h + 4, 4);
	REQUIRE(memcmp(h + 8, "WAVEfmt ", 8) == 0, EPROTO);
	hdr_len = get_le(h + 16, 4);
	tag = (uint16_t)get_le(h + 20, 2);
	chans = (uint16_t)get_le(h + 22, 2);
	rate = get_le(h + 24, 4);
	byte_rate = get_le(h + 28, 4);
	align = (uint16_t)get_le(h + 32, 2);
	bits = (uint16_t)get_le(h + 34, 2);
	REQUIRE(memcmp(h + 36, "data", 4) == 0, EPROTO);
	data_len = get_le(h + 40, 4);

	/* checks of :855-863, same 32-bit wrap-around */
	REQUIRE(riff_len >= (uint32_t)(BJXA_HEADER_SIZE_RIFF - 8) + data_len,
	    EPROTO);
	REQUIRE(hdr_len == 16, EPROTO);
	REQUIRE(tag == 1, EPROTO);
	REQUIRE(chans == 1 || chans == 2, EPROTO);
	REQUIRE(rate > 0 && rate < UINT16_MAX, EPROTO);
	REQUIRE(align == chans * 2u, EPROTO);
	REQUIRE(byte_rate == (uint32_t)(rate * align), EPROTO);
	REQUIRE(data_len % align == 0, EPROTO);
	REQUIRE(bits == 16, EPROTO);

	memset(&out, 0, sizeof out);
	out.data_len_pcm = data_len;
	out.samples_rate = (uint16_t)rate;
	out.sample_bits = 16;
	out.channels = (uint8_t)chans;
	*fmt = out;
	return (BJXA_HEADER_SIZE_RIFF);
}

ssize_t
bjxa_fread_riff_header(bjxa_format_t *fmt, FILE *file)
{
	uint8_t buf[BJXA_HEADER_SIZE_RIFF];
	ssize_t ret;

	NEED_PTR(fmt);
	NEED_PTR(file);
	if (read_all(buf, sizeof buf, file) < 0)
		return (-1);
	ret = bjxa_parse_riff_header(fmt, buf, sizeof buf);
	assert(ret >= 0 || (errno != EINVAL && errno != ENOBUFS));
	return (ret);
}

ssize_t
bjxa_dump_riff_header(bjxa_decoder_t *dec, void *dst, size_t len)
{
	bjxa_format_t fmt;
	uint8_t *p = dst;

	NEED_OBJ(dec, DEC_MAGIC);
	NEED_PTR(dst);
	REQUIRE(len >= BJXA_HEADER_SIZE_RIFF, ENOBUFS);
	if (bjxa_decode_format(dec, &fmt) < 0)
		return (-1);

	p = put_tag(p, "RIFF");
	p = put_le(p, BJXA_HEADER_SIZE_RIFF - 8 + fmt.data_len_pcm, 4);
	p = put_tag(p, "WAVEfmt ");
	p = put_le(p, 16, 4);
	p = put_le(p, 1, 2);			/* PCM */
	p = put_le(p, fmt.channels, 2);
	p = put_le(p, fmt.samples_rate, 4);
	p = put_le(p, (uint32_t)fmt.samples_rate * fmt.block_size_pcm /
	    XA_FRAMES, 4);
	p = put_le(p, fmt.channels * fmt.sample_bits / 8u, 2);
	p = put_le(p, fmt.sample_bits, 2);
	p = put_tag(p, "data");
	(void)put_le(p, fmt.data_len_pcm, 4);
	return (BJXA_HEADER_SIZE_RIFF);
}

ssize_t
bjxa_fwrite_riff_header(bjxa_decoder_t *dec, FILE *file)
{
	uint8_t buf[BJXA_HEADER_SIZE_RIFF];

	NEED_OBJ(dec, DEC_MAGIC);
	NEED_PTR(file);
	if (bjxa_dump_riff_header(dec, buf, sizeof buf) < 0)
		return (-1);
	if (fwrite(buf, sizeof buf, 1, file) != 1)
		return (-1);
	return (BJXA_HEADER_SIZE_RIFF);
}

int
bjxa_dump_pcm(void *dst, const int16_t *src, size_t len)
{
	uint8_t *p = dst;
	size_t i;

	NEED_PTR(dst);
	NEED_PTR(src);
	REQUIRE(len > 0, ENOBUFS);
	REQUIRE((len & 1) == 0, ENOBUFS);
	for (i = 0; i < len / 2; i++)
		p = put_le(p, (uint16_t)src[i], 2);
	return (0);
}

int
bjxa_fwrite_pcm(const int16_t *src, size_t len, FILE *file)
{
	uint8_t buf[8192];

	NEED_PTR(src);
	NEED_PTR(file);
	REQUIRE(len > 0, ENOBUFS);
	REQUIRE((len & 1) == 0, ENOBUFS);
	while (len > 0) {
		size_t n = len < sizeof buf ? len : sizeof buf;
		(void)bjxa_dump_pcm(buf, src, n);
		if (fwrite(buf, n, 1, file) != 1)
			return (-1);
		src += n / 2;
		len -= n;
	}
	return (0);
}

/* ---- encode (src/libbjxa.c:693-819) ---------------------------------- */

int
bjxa_encode_init(bjxa_encoder_t *enc, bjxa_format_t *fmt, uint8_t bits)
{
	bjxa_encoder_t tmp;

	NEED_OBJ(enc, ENC_MAGIC);
	NEED_PTR(fmt);
	REQUIRE(fmt->sample_bits == 16, EINVAL);
	REQUIRE(bits == 4 || bits == 6 || bits == 8, EINVAL);

	memset(&tmp, 0, sizeof tmp);
	tmp.bits = bits;
	tmp.channels = fmt->channels;
	REQUIRE(tmp.channels == 1 || tmp.channels == 2, EPROTO);
	tmp.samples = fmt->data_len_pcm / (tmp.channels * 2u);
	tmp.rate = fmt->samples_rate;
	REQUIRE(tmp.samples > 0, EPROTO);
	REQUIRE(tmp.rate > 0, EPROTO);
	REQUIRE(fmt->data_len_pcm % tmp.samples == 0, EPROTO);

	tmp.block_size = (uint8_t)(bits * 4 + 1);
	fmt->block_size_xa = (uint8_t)(tmp.block_size * tmp.channels);
	fmt->block_size_pcm = (uint8_t)(XA_FRAMES * tmp.channels * 2u);
	fmt->blocks = (tmp.samples + XA_FRAMES - 1) / XA_FRAMES;
	tmp.data_len = fmt->blocks * fmt->block_size_xa;

	tmp.left = *fmt;
	tmp.magic = ENC_MAGIC;
	tmp.gpu = enc->gpu;
	*enc = tmp;
	return (0);
}

int
bjxa_encode_format(bjxa_encoder_t *enc, bjxa_format_t *fmt)
{
	NEED_OBJ(enc, ENC_MAGIC);
	NEED_PTR(fmt);
	REQUIRE(enc->block_size != 0, EINVAL);

	fmt->data_len_pcm = enc->samples * enc->channels * 2u;
	fmt->samples_rate = enc->rate;
	fmt->sample_bits = enc->bits;
	fmt->channels = enc->channels;
	fmt->block_size_xa = (uint8_t)(enc->block_size * enc->channels);
	fmt->block_size_pcm = (uint8_t)(XA_FRAMES * enc->channels * 2u);
	fmt->blocks = enc->data_len / fmt->block_size_xa;
	assert(fmt->blocks * fmt->block_size_xa == enc->data_len);
	return (0);
}

int
bjxa_encode(bjxa_encoder_t *enc, void *dst, size_t dst_len, const void *src,
    size_t src_len)
{
	bjxa_format_t *f;
	uint64_t n, take, frames;

	NEED_OBJ(enc, ENC_MAGIC);
	NEED_PTR(dst);
	NEED_PTR(src);
	f = &enc->left;
	REQUIRE(f->sample_bits == 16, EINVAL);
	REQUIRE(f->blocks > 0, EPROTO);
	REQUIRE(dst_len >= f->block_size_xa, ENOBUFS);
	REQUIRE(src_len >= f->block_size_pcm, ENOBUFS);

	/* mirror of the loop at :787-816 */
	n = f->blocks;
	if (dst_len / f->block_size_xa < n)
		n = dst_len / f->block_size_xa;
	if (src_len < f->data_len_pcm && src_len / f->block_size_pcm < n)
		n = src_len / f->block_size_pcm;
	take = n * f->block_size_pcm;
	if (take > f->data_len_pcm)
		take = f->data_len_pcm;
	/* frames per block = PCM bytes of that block / frame size; only the
	 * last block of the stream can be short */
	frames = (n - 1) * XA_FRAMES + (take - (n - 1) * f->block_size_pcm) /
	    (enc->channels * 2u);

	if (!on_gpu(BJXA_HIP_OFFLOAD_ENCODE, n)) {
		(void)bjxa__cpu_encode(src, frames, enc->bits, enc->channels,
		    dst);
	} else {
		if (enc->gpu == NULL && (enc->gpu = bjxa__gpu_new()) == NULL)
			return (-1);
		if (bjxa__gpu_encode(enc->gpu, src, frames, enc->bits,
		    enc->channels, dst) < 0)
			return (-1);
	}
	f->blocks -= (uint32_t)n;
	f->data_len_pcm -= (uint32_t)take;
	return ((int)n);
}

/* ---- many files in one batched pass (LIBBJXA_HIP_0.1) ----------------- */

/*
 * bjxa_hip_decode_files: decode n complete XA files (32-byte header +
 * blocks) held in host memory into n complete WAV files -- the 44-byte RIFF
 * header of bjxa_dump_riff_header followed by the PCM (host order, which
 * is little-endian on the hosts this library targets, so bjxa_dump_pcm's
 * conversion is the identity) -- with one batched GPU pass over all of
 * them.  status[i] is 0 or the errno file i failed with: EPROTO for a bad
 * header or a block profile with gain >= 5 (the WAV then holds the header
 * and the PCM before that block), ENOBUFS for an input shorter than its
 * header announces or an output smaller than 44 + data_len_pcm.  Returns
 * the number of files decoded completely, or -1 with errno (EFAULT,
 * EINVAL, or the device's ENODEV/ENOMEM/EIO) when the batch itself fails.
 */
int
bjxa_hip_decode_files(const void *const *xa, const size_t *xa_len,
    void *const *wav, const size_t *wav_len, int *status, uint32_t n)
{
	struct bjxa__job *jobs;
	uint32_t *which, nj = 0;
	int done = 0;

	NEED_PTR(xa);
	NEED_PTR(xa_len);
	NEED_PTR(wav);
	NEED_PTR(wav_len);
	NEED_PTR(status);
	REQUIRE(n > 0, EINVAL);
	jobs = calloc(n, sizeof *jobs);
	which = calloc(n, sizeof *which);
	if (jobs == NULL || which == NULL) {
		free(jobs);
		free(which);
		FAIL(ENOMEM);
	}
	for (uint32_t i = 0; i < n; i++) {
		const uint8_t *h = xa[i];
		bjxa_decoder_t d;
		bjxa_format_t f;

		status[i] = 0;
		if (h == NULL || wav[i] == NULL) {
			status[i] = EFAULT;
			continue;
		}
		if (xa_len[i] < BJXA_HEADER_SIZE_XA) {
			status[i] = ENOBUFS;
			continue;
		}
		/* a stereo payload of an odd number of channel blocks would
		 * trip the format assertion (:597): refuse it here instead */
		if (h[15] == 2 && (h[14] == 4 || h[14] == 6 || h[14] == 8) &&
		    get_le(h + 4, 4) % (2u * (h[14] * 4u + 1u)) != 0) {
			status[i] = EPROTO;
			continue;
		}
		memset(&d, 0, sizeof d);
		d.magic = DEC_MAGIC;
		if (bjxa_parse_header(&d, h, xa_len[i]) < 0) {
			status[i] = errno;
			continue;
		}
		dec_format(&d, &f);
		if (xa_len[i] < BJXA_HEADER_SIZE_XA + (size_t)f.blocks *
		    f.block_size_xa || wav_len[i] < BJXA_HEADER_SIZE_RIFF +
		    (size_t)f.data_len_pcm) {
			status[i] = ENOBUFS;
			continue;
		}
		(void)bjxa_dump_riff_header(&d, wav[i], BJXA_HEADER_SIZE_RIFF);
		jobs[nj].src = h + BJXA_HEADER_SIZE_XA;
		jobs[nj].dst = (uint8_t *)wav[i] + BJXA_HEADER_SIZE_RIFF;
		jobs[nj].dst_bytes = f.data_len_pcm;
		jobs[nj].eblocks = f.blocks;
		jobs[nj].bits = d.bits;
		jobs[nj].ch = d.channels;
		memcpy(jobs[nj].state, d.state, sizeof d.state);
		which[nj++] = i;
	}
	if (nj > 0 && bjxa__gpu_decode_many(jobs, nj) < 0) {
		const int e = errno;
		free(jobs);
		free(which);
		FAIL(e);
	}
	for (uint32_t k = 0; k < nj; k++)
		if (jobs[k].err_cb != 0xffffffffu)
			status[which[k]] = EPROTO;
	for (uint32_t i = 0; i < n; i++)
		done += status[i] == 0;
	free(jobs);
	free(which);
	return (done);
}
