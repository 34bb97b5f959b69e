/*
 * melpe.h -- drop-in replacement for the reference codec's public header
 * (reference melpe/melpe.h:1-19).  Same four symbols, same single-stream
 * semantics, so PairPhone's tx.c / rx.c and melpe_enc.c / melpe_dec.c relink
 * against libmelpe_amd.so unchanged.
 *
 *   melpe_n   melpe/melpe.c:63   denoise 180 samples in place (NPP only)
 *   melpe_i   melpe/melpe.c:72   initialise the 1200 bps codec
 *   melpe_a   melpe/melpe.c:91   540 samples -> 81 bits (11 bytes); sp is
 *                                overwritten with the NPP output, as in the
 *                                reference (melpe/melpe.c:94-96)
 *   melpe_s   melpe/melpe.c:102  11 bytes -> 540 samples
 *
 * The 2400 bps entry points the reference declares but never defines
 * (melpe/melpe.c:57-58) are provided as their names and the reference's
 * RATE2400 code define them:
 *   melpe_i2  initialise at 2400 bps (melpe_i with rate = RATE2400)
 *   melpe_al  180 samples -> 54 bits (7 bytes), sp overwritten with the NPP
 *             output; after melpe_i2, melpe_s decodes 7 bytes -> 180 samples
 *
 * As in the reference, the encoder and decoder of the one process-global
 * instance share melp_par / quant_par / chbuf (melpe/global.c:28-37), so an
 * interleaved melpe_a / melpe_s sequence (PairPhone's duplex pp) decodes as
 * the reference does.  The batched ABI (melpe_batch.h) keeps them separate
 * per channel, i.e. standalone melpe_enc / melpe_dec semantics.
 * The functions compute on the GPU; with no usable GPU they print an error
 * and abort() -- there is no CPU fallback.
 */
#ifndef MELPE_AMD_MELPE_H
#define MELPE_AMD_MELPE_H

#ifdef __cplusplus
extern "C" {
#endif

void melpe_n(short *sp);
void melpe_i(void);
void melpe_a(unsigned char *buf, short *sp);
void melpe_s(short *sp, unsigned char *buf);
void melpe_i2(void);
void melpe_al(unsigned char *buf, short *sp);

#ifdef __cplusplus
}
#endif

#endif
