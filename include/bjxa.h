/*
 * bjxa.h -- public C API of the MI355X libbjxa (drop-in for the reference
 * library's src/bjxa.h:18-65; same prototypes, same bjxa_format_t layout,
 * same symbol versions LIBBJXA_0.1 / LIBBJXA_0.5, src/libbjxa.map:16-47).
 *
 * As with the reference header, callers include <stdint.h>, <stdio.h> and
 * <sys/types.h> (for ssize_t) first.  Every entry point returns -1 (or
 * NULL) and sets errno on failure; see bjxa.3 for the errno contract.
 *
 * Decoding and encoding run on the GPU (hand-written gfx950 kernels) for
 * calls of at least the offload threshold (bjxa_hip.h,
 * bjxa_hip_offload_threshold) and on the calling thread's core below it and
 * on hosts without a usable GPU; both give the reference's bytes, block
 * counts, errno and carried state.  The framing functions are host C.
 */
#ifndef BJXA_H_INCLUDED
#define BJXA_H_INCLUDED

#ifdef __cplusplus
extern "C" {
#endif

/* on-disk header sizes: XA "KWD1" header and canonical 44-byte WAVE */
#define BJXA_HEADER_SIZE_XA	32
#define BJXA_HEADER_SIZE_RIFF	44

/* opaque codec objects (one thread at a time per object) */
typedef struct bjxa_decoder bjxa_decoder_t;
typedef struct bjxa_encoder bjxa_encoder_t;

/*
 * Stream description exchanged with callers.  16 bytes; member offsets
 * 0/4/8/9/10/12/13 as in the reference.
 */
typedef struct {
	uint32_t	data_len_pcm;	/* PCM bytes still to produce/consume */
	uint32_t	blocks;		/* effective blocks still to process */
	uint8_t		block_size_pcm;	/* 64 * channels */
	uint8_t		block_size_xa;	/* (bits * 4 + 1) * channels */
	uint16_t	samples_rate;
	uint8_t		sample_bits;	/* 16 for PCM; XA bits for encoders */
	uint8_t		channels;	/* 1 or 2 */
} bjxa_format_t;

/* --- decoder (LIBBJXA_0.1) ------------------------------------------ */

/* allocate / release; release zeroes the object and NULLs *decp */
bjxa_decoder_t *bjxa_decoder(void);
int bjxa_free_decoder(bjxa_decoder_t **decp);

/* load a 32-byte XA header (state replaced only on success) */
ssize_t bjxa_parse_header(bjxa_decoder_t *dec, const void *src, size_t len);
ssize_t bjxa_fread_header(bjxa_decoder_t *dec, FILE *file);

/* describe the remaining stream */
int bjxa_decode_format(bjxa_decoder_t *dec, bjxa_format_t *fmt);

/*
 * Decode as many effective blocks as fit both buffers (at least one full
 * block each); returns the number decoded.  Predictor state and remaining
 * counts persist across calls.
 */
int bjxa_decode(bjxa_decoder_t *dec, void *dst, size_t dst_len,
    const void *src, size_t src_len);

/* 44-byte RIFF/WAVE header for the decoder's stream */
ssize_t bjxa_dump_riff_header(bjxa_decoder_t *dec, void *dst, size_t len);
ssize_t bjxa_fwrite_riff_header(bjxa_decoder_t *dec, FILE *file);

/* host-endian int16 samples -> little-endian bytes */
int bjxa_dump_pcm(void *dst, const int16_t *src, size_t len);
int bjxa_fwrite_pcm(const int16_t *src, size_t len, FILE *file);

/* --- encoder (LIBBJXA_0.5) ------------------------------------------ */

bjxa_encoder_t *bjxa_encoder(void);
int bjxa_free_encoder(bjxa_encoder_t **encp);

/* set up from a PCM description and a code width of 4, 6 or 8 bits */
int bjxa_encode_init(bjxa_encoder_t *enc, bjxa_format_t *fmt, uint8_t bits);

/* read a 44-byte RIFF/WAVE header into a format description */
ssize_t bjxa_parse_riff_header(bjxa_format_t *fmt, const void *src,
    size_t len);
ssize_t bjxa_fread_riff_header(bjxa_format_t *fmt, FILE *file);

int bjxa_encode_format(bjxa_encoder_t *enc, bjxa_format_t *fmt);
int bjxa_encode(bjxa_encoder_t *enc, void *dst, size_t dst_len,
    const void *src, size_t src_len);

/* 32-byte XA header for the encoder's stream */
ssize_t bjxa_dump_header(bjxa_encoder_t *enc, void *dst, size_t len);
ssize_t bjxa_fwrite_header(bjxa_encoder_t *enc, FILE *file);

#ifdef __cplusplus
}
#endif

#endif /* BJXA_H_INCLUDED */
