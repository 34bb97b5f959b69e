/*
 * ref_vad.c -- TEST INFRASTRUCTURE ONLY (oracle; never linked into the
 * product).  Drives the reference's AMR VAD option 2 (vad/vad2.c, compiled
 * where it lies with its basic ops by oracle/Makefile into
 * oracle/_ref/libref_vad.so) the way PairPhone's TX path does: a fresh
 * vad2_reset state per channel (the reset melpe_enc.c:36 omits, SURVEY.md
 * §8(c).6), then per superframe the six vad2 calls at offsets 10, 100, ...,
 * 460 (tx.c:234-239, melpe_enc.c:48-53), votes = the sum of the decisions.
 */
#include <stdint.h>
#include <stddef.h>
#include "typedef.h"
#include "vad2.h"

/* sp: C x (nsf*540) int16 channel-major; votes: C x nsf */
int ref_vad(const int16_t *sp, uint8_t *votes, int channels, int nsf)
{
	for (int c = 0; c < channels; c++) {
		vadState2 st;
		vad2_reset(&st);
		for (int k = 0; k < nsf; k++) {
			Word16 *x = (Word16 *) (sp + ((size_t) c * nsf + k) * 540);
			int n = 0;
			for (int w = 0; w < 6; w++)
				n += vad2(x + 10 + 90 * w, &st);
			votes[(size_t) c * nsf + k] = (uint8_t) n;
		}
	}
	return 0;
}
