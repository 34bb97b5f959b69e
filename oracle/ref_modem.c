/*
 * ref_modem.c -- harness around the REFERENCE pseudo-voice modem
 * (modem/modem.c: Modulate :136, Demodulate :186, compiled where it lies by
 * oracle/Makefile; TEST INFRASTRUCTURE ONLY).  The modem keeps its state in
 * file statics (modem.c:48-73), so one process = one channel, as PairPhone
 * runs it.
 *
 *   ref_modem mod   <in.bits> <out.pcm>
 *       Modulate each 11-byte packet of in.bits (tx.c:271) -> 3240 int16
 *       samples per packet.
 *   ref_modem demod <in.pcm> <calls> <out.dat>
 *       Demodulate as rx.c:294-297 drives it: pos starts at 0, each call
 *       gets samples + pos and pos advances by the return value; the same
 *       12-byte buf persists across calls (rx.c keeps it).  Per call writes
 *       the 12 bytes of buf after the call and the int32 return value.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "modem.h"

static long fsize(FILE *f)
{
	long n;
	fseek(f, 0, SEEK_END);
	n = ftell(f);
	fseek(f, 0, SEEK_SET);
	return n;
}

int main(int argc, char **argv)
{
	if (argc == 4 && !strcmp(argv[1], "mod")) {
		FILE *fi = fopen(argv[2], "rb"), *fo = fopen(argv[3], "wb");
		unsigned char pk[11];
		short pcm[3240];
		if (!fi || !fo)
			return 2;
		while (fread(pk, 1, 11, fi) == 11) {
			int n = Modulate(pk, pcm);
			if (n != 3240)
				return 3;
			fwrite(pcm, 2, 3240, fo);
		}
		fclose(fi);
		fclose(fo);
		return 0;
	}
	if (argc == 5 && !strcmp(argv[1], "demod")) {
		FILE *fi = fopen(argv[2], "rb"), *fo = fopen(argv[4], "wb");
		long calls = atol(argv[3]), n, pos = 0, k;
		short *pcm;
		unsigned char buf[12];
		if (!fi || !fo)
			return 2;
		n = fsize(fi) / 2;
		pcm = (short *) calloc(n, 2);
		if (fread(pcm, 2, n, fi) != (size_t) n)
			return 4;
		memset(buf, 0, sizeof buf);
		for (k = 0; k < calls; k++) {
			int32_t r;
			if (pos + 1080 > n)
				return 5;	/* rx.c:246 needs 180*6 samples */
			r = Demodulate(pcm + pos, buf);
			pos += r;
			fwrite(buf, 1, 12, fo);
			fwrite(&r, 4, 1, fo);
		}
		free(pcm);
		fclose(fi);
		fclose(fo);
		return 0;
	}
	fprintf(stderr, "usage: ref_modem mod <bits> <pcm> | demod <pcm> <calls> <out>\n");
	return 1;
}
