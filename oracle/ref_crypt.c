/*
 * ref_crypt.c -- TEST INFRASTRUCTURE ONLY (oracle; never linked into the
 * product).  Exposes PairPhone's voice-frame crypt through the reference's
 * own Keccak sponge (crypto/sponge.c, compiled where it lies by
 * oracle/Makefile into oracle/_ref/libref_crypt.so).
 *
 * VoiceEnc / VoiceDec are `static` in crp.c (crp.c:986-1027), whose other
 * dependencies (curve, havege, golay FEC, the call state machine) are not
 * needed for this step, so their ten lines are restated here call for call:
 * IntToBytes(udata, cnt) (crp.c:322-327), Sponge_init(0,0,0,0),
 * Sponge_data(counter, 4), Sponge_data(key, 16), Sponge_finalize(udata, 11),
 * udata[10] &= 1, pkt ^= udata; VoiceDec inverts first when finv < 0.
 */
#include <stdint.h>
#include <string.h>
#include "sponge.h"

static void int_to_bytes(unsigned char *b, unsigned int v)
{
	b[0] = v & 0xFF;
	b[1] = (v >> 8) & 0xFF;
	b[2] = (v >> 16) & 0xFF;
	b[3] = (v >> 24) & 0xFF;
}

/* crp.c:986-1000 (dir 0) and :1004-1027 (dir 1), one packet */
static void voice_crypt_one(unsigned char *pkt, unsigned int cnt, const unsigned char *key,
			    int dir, int finv_negative)
{
	KECCAK512_DATA spng;
	unsigned char udata[16];
	int i;
	if (dir && finv_negative) {
		for (i = 0; i < 10; i++)
			pkt[i] ^= 0xFF;
		pkt[10] ^= 1;
	}
	int_to_bytes(udata, cnt);
	Sponge_init(&spng, 0, 0, 0, 0);
	Sponge_data(&spng, udata, 4, 0, SP_NORMAL);
	Sponge_data(&spng, key, 16, 0, SP_NORMAL);
	Sponge_finalize(&spng, udata, 11);
	udata[10] &= 0x01;
	for (i = 0; i < 11; i++)
		pkt[i] ^= udata[i];
}

/* same layout as melpe_voice_crypt_host (include/melpe_batch.h) */
int ref_voice_crypt(unsigned char *pkts, const uint32_t *counters, const unsigned char *keys,
		    const uint8_t *invert, int channels, int packets, int dir)
{
	for (int c = 0; c < channels; c++)
		for (int k = 0; k < packets; k++)
			voice_crypt_one(pkts + ((size_t) c * packets + k) * 11,
					counters[c] + (unsigned int) k, keys + 16 * (size_t) c, dir,
					invert ? invert[c] != 0 : 0);
	return 0;
}
