/*
 * ref_tool.c -- oracle harness around the REFERENCE MELPe codec
 * (TEST INFRASTRUCTURE ONLY: never linked into the product library).
 *
 * Links oracle/_ref/libmelpe_ref.a, which oracle/Makefile compiles from
 * /root/reference/melpe/*.c unchanged, and drives it exactly the way the
 * reference's own harnesses do:
 *   - encode: melpe/encoder.c:29-45 (melpe_i once, melpe_a per 540 samples,
 *     a final partial superframe zero-padded);
 *   - decode: melpe/decoder.c:27-31 (melpe_i once, melpe_s per 11 bytes);
 *   - npp:    melpe/melpe.c:63-67 (melpe_n per 180 samples, after melpe_i).
 * The reference keeps all codec state in process globals
 * (melpe/global.c:20-53 plus function statics), so every channel is run in a
 * freshly forked child process: that is the only true reset.
 *
 * Commands (PCM is raw little-endian int16, 8 kHz):
 *   gen    <seed> <channel> <nsamples> <out.pcm>
 *   enc    <in.pcm> <out.bits> [<dump.bin>]
 *   dec    <in.bits> <out.pcm> [<dump.bin>]
 *   npp    <in.pcm> <out.pcm>
 *   duplex <in.pcm> <in.bits> <out.bits> <out.pcm>
 *          one process running melpe_a (on in.pcm) and melpe_s (on in.bits)
 *          alternately, superframe by superframe, as a PairPhone endpoint
 *          does: the two share melp_par / quant_par / chbuf
 *   encgen <seed> <ch0> <nch> <nsf> <out.bits> [<out.npp.pcm>]
 *          channel c = synth_mix(seed, c) signal, nsf superframes each,
 *          bitstreams concatenated channel-major (nch*nsf*11 bytes)
 *   decgen <in.bits> <nch> <nsf> <out.pcm>
 *          decodes nch independent channel bitstreams (channel-major)
 *   enc24gen <seed> <ch0> <nch> <nfr> <out.bits> [<out.npp.pcm>]
 *   dec24gen <in.bits> <nch> <nfr> <out.pcm>
 *          the 2400 bps MELP path, which the reference
 *          compiles but never reaches: melpe_i pins rate = RATE1200
 *          (melpe/melpe.c:76) and the 2400 entry points melpe_i2 / melpe_al
 *          it declares (melpe/melpe.c:57-58) have no bodies.  The harness
 *          sets the globals as melpe_i would for RATE2400 (frameSize =
 *          FRAME, 54 bits in 7 bytes) and calls the reference's own
 *          npp + analysis per 180-sample frame (melpe_a's body for one
 *          frame) and synthesis per 7-byte frame (melpe_s's body)
 *   jobs   <n>   (prefix option: max parallel children, default 8)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <unistd.h>
#include <sys/wait.h>

#include "sc1200.h"
#include "global.h"
#include "melpe.h"
#include "npp.h"
#include "synth.h"

extern int16_t mode, chwordsize, bitBufSize, bitBufSize12, bitBufSize24;

extern struct melp_param melp_par[];
extern struct quant_param quant_par;
extern unsigned char chbuf[];

static int g_jobs = 8;

static void *read_file(const char *path, long *len)
{
	FILE *f = fopen(path, "rb");
	void *buf;
	if (!f) {
		perror(path);
		exit(2);
	}
	fseek(f, 0, SEEK_END);
	*len = ftell(f);
	fseek(f, 0, SEEK_SET);
	buf = malloc(*len + 4096);
	memset(buf, 0, *len + 4096);
	if (*len && fread(buf, 1, *len, f) != (size_t) *len) {
		perror("fread");
		exit(2);
	}
	fclose(f);
	return buf;
}

/* quant_par without the pointer members, as plain int16 words */
static void dump_quant(FILE *f)
{
	int16_t w[30];
	int k = 0, i, j;
	w[k++] = quant_par.pitch_index;
	for (i = 0; i < NF; i++)
		for (j = 0; j < MAX_LSF_STAGE; j++)
			w[k++] = quant_par.lsf_index[i][j];
	for (i = 0; i < NUM_GAINFR; i++)
		w[k++] = quant_par.gain_index[i];
	for (i = 0; i < NF; i++)
		w[k++] = quant_par.jit_index[i];
	for (i = 0; i < NF; i++)
		w[k++] = quant_par.bpvc_index[i];
	w[k++] = quant_par.fs_index;
	for (i = 0; i < NF; i++)
		w[k++] = quant_par.uv_flag[i];
	for (i = 0; i < MSVQ_STAGES; i++)
		w[k++] = quant_par.msvq_index[i];
	w[k++] = quant_par.fsvq_index;
	fwrite(w, 2, 30, f);
}

/* Encode a whole PCM buffer of n samples like melpe/encoder.c. */
static long encode_buffer(const int16_t *pcm, long n, unsigned char *bits,
			  int16_t *npp_out, FILE *dump)
{
	short sp[BLOCK];
	long pos = 0, nsf = 0;
	unsigned char pad = 0;
	melpe_i();
	while (pos < n) {
		long take = n - pos < BLOCK ? n - pos : BLOCK;
		memset(sp, 0, sizeof(sp));
		memcpy(sp, pcm + pos, take * 2);
		melpe_a(bits + nsf * 11, sp);
		if (npp_out)
			memcpy(npp_out + nsf * BLOCK, sp, sizeof(sp));
		if (dump) {
			fwrite(melp_par, sizeof(struct melp_param), NF, dump);
			dump_quant(dump);
			fwrite(bits + nsf * 11, 1, 11, dump);
			fwrite(&pad, 1, 1, dump);
			fwrite(sp, 2, BLOCK, dump);
		}
		pos += take;
		nsf++;
	}
	return nsf;
}

static void decode_buffer(const unsigned char *bits, long nsf, int16_t *pcm,
			  FILE *dump)
{
	long k;
	unsigned char buf[11];
	melpe_i();
	for (k = 0; k < nsf; k++) {
		memcpy(buf, bits + k * 11, 11);
		melpe_s(pcm + k * BLOCK, buf);
		if (dump)
			fwrite(melp_par, sizeof(struct melp_param), NF, dump);
	}
}

/* RATE2400 initialisation: melpe_i (melpe/melpe.c:72-88) with rate =
 * RATE2400 and one-frame blocks */
static void init2400(void)
{
	mode = ANA_SYN;
	rate = RATE2400;
	frameSize = (int16_t) FRAME;
	chwordsize = 8;
	bitNum12 = 81;
	bitNum24 = 54;
	bitBufSize12 = 11;
	bitBufSize24 = 7;
	bitBufSize = bitBufSize24;
	melp_ana_init();
	melp_syn_init();
}

/* 2400 bps encode of n samples: per 180-sample frame npp in place, then
 * analysis (one frame at RATE2400), 7 bytes of chbuf out */
static long encode2400(const int16_t *pcm, long n, unsigned char *bits, int16_t *npp_out)
{
	short sp[FRAME];
	long k, nfr = n / FRAME;
	init2400();
	for (k = 0; k < nfr; k++) {
		memcpy(sp, pcm + k * FRAME, sizeof(sp));
		npp(sp, sp);
		analysis(sp, melp_par);
		memcpy(bits + k * 7, chbuf, 7);
		if (npp_out)
			memcpy(npp_out + k * FRAME, sp, sizeof(sp));
	}
	return nfr;
}

static void decode2400(const unsigned char *bits, long nfr, int16_t *pcm)
{
	long k;
	init2400();
	for (k = 0; k < nfr; k++) {
		memcpy(chbuf, bits + k * 7, 7);
		synthesis(melp_par, pcm + k * FRAME);
	}
}

/* Runs fn(c) for c in [0,n) in forked children, at most g_jobs at a time. */
static void run_children(long n, void (*fn)(long, void *), void *arg)
{
	long c, running = 0;
	int status;
	for (c = 0; c < n; c++) {
		pid_t pid;
		if (running >= g_jobs) {
			wait(&status);
			if (!WIFEXITED(status) || WEXITSTATUS(status)) {
				fprintf(stderr, "child failed\n");
				exit(3);
			}
			running--;
		}
		pid = fork();
		if (pid < 0) {
			perror("fork");
			exit(3);
		}
		if (pid == 0) {
			fn(c, arg);
			_exit(0);
		}
		running++;
	}
	while (running > 0) {
		wait(&status);
		if (!WIFEXITED(status) || WEXITSTATUS(status)) {
			fprintf(stderr, "child failed\n");
			exit(3);
		}
		running--;
	}
}

struct encgen_arg {
	uint32_t seed;
	long ch0, nsf;
	const char *out_bits, *out_npp;
};

static void write_at(const char *path, long off, const void *data, long len)
{
	FILE *f = fopen(path, "r+b");
	if (!f) {
		perror(path);
		_exit(4);
	}
	fseek(f, off, SEEK_SET);
	fwrite(data, 1, len, f);
	fclose(f);
}

static void encgen_one(long c, void *varg)
{
	struct encgen_arg *a = (struct encgen_arg *) varg;
	long n = a->nsf * BLOCK;
	int16_t *pcm = (int16_t *) calloc(n, 2);
	int16_t *npp = (int16_t *) calloc(n, 2);
	unsigned char *bits = (unsigned char *) calloc(a->nsf, 11);
	synth_state st;
	synth_init(&st, synth_mix(a->seed, (uint32_t) (a->ch0 + c)));
	synth_block(&st, pcm, (int) n);
	encode_buffer(pcm, n, bits, npp, NULL);
	write_at(a->out_bits, c * a->nsf * 11, bits, a->nsf * 11);
	if (a->out_npp)
		write_at(a->out_npp, c * n * 2, npp, n * 2);
}

struct decgen_arg {
	const unsigned char *bits;
	long nsf;
	const char *out;
};

static void decgen_one(long c, void *varg)
{
	struct decgen_arg *a = (struct decgen_arg *) varg;
	int16_t *pcm = (int16_t *) calloc(a->nsf * BLOCK, 2);
	decode_buffer(a->bits + c * a->nsf * 11, a->nsf, pcm, NULL);
	write_at(a->out, c * a->nsf * BLOCK * 2, pcm, a->nsf * BLOCK * 2);
}

static void enc24gen_one(long c, void *varg)
{
	struct encgen_arg *a = (struct encgen_arg *) varg;	/* nsf = frames */
	long n = a->nsf * FRAME;
	int16_t *pcm = (int16_t *) calloc(n + 256, 2);
	int16_t *npp_o = (int16_t *) calloc(n, 2);
	unsigned char *bits = (unsigned char *) calloc(a->nsf, 7);
	synth_state st;
	synth_init(&st, synth_mix(a->seed, (uint32_t) (a->ch0 + c)));
	synth_block(&st, pcm, (int) n);
	encode2400(pcm, n, bits, npp_o);
	write_at(a->out_bits, c * a->nsf * 7, bits, a->nsf * 7);
	if (a->out_npp)
		write_at(a->out_npp, c * n * 2, npp_o, n * 2);
}

static void dec24gen_one(long c, void *varg)
{
	struct decgen_arg *a = (struct decgen_arg *) varg;	/* nsf = frames */
	int16_t *pcm = (int16_t *) calloc(a->nsf * FRAME, 2);
	decode2400(a->bits + c * a->nsf * 7, a->nsf, pcm);
	write_at(a->out, c * a->nsf * FRAME * 2, pcm, a->nsf * FRAME * 2);
}

static void make_file(const char *path, long len)
{
	FILE *f = fopen(path, "wb");
	if (!f) {
		perror(path);
		exit(2);
	}
	if (len > 0) {
		fseek(f, len - 1, SEEK_SET);
		fputc(0, f);
	}
	fclose(f);
}

int main(int argc, char **argv)
{
	if (argc >= 3 && !strcmp(argv[1], "jobs")) {
		g_jobs = atoi(argv[2]);
		if (g_jobs < 1)
			g_jobs = 1;
		argv += 2;
		argc -= 2;
	}
	if (argc < 2) {
		fprintf(stderr, "usage: see header of oracle/ref_tool.c\n");
		return 1;
	}
	if (!strcmp(argv[1], "gen") && argc == 6) {
		long n = atol(argv[4]);
		int16_t *pcm = (int16_t *) calloc(n, 2);
		synth_state st;
		FILE *f;
		synth_init(&st, synth_mix((uint32_t) strtoul(argv[2], 0, 0),
					  (uint32_t) strtoul(argv[3], 0, 0)));
		synth_block(&st, pcm, (int) n);
		f = fopen(argv[5], "wb");
		fwrite(pcm, 2, n, f);
		fclose(f);
		return 0;
	}
	if (!strcmp(argv[1], "enc") && (argc == 4 || argc == 5)) {
		long len, nsf;
		int16_t *pcm = (int16_t *) read_file(argv[2], &len);
		unsigned char *bits = (unsigned char *) malloc((len / 2 / BLOCK + 2) * 11);
		FILE *dump = argc == 5 ? fopen(argv[4], "wb") : NULL;
		FILE *f;
		nsf = encode_buffer(pcm, len / 2, bits, NULL, dump);
		f = fopen(argv[3], "wb");
		fwrite(bits, 11, nsf, f);
		fclose(f);
		if (dump)
			fclose(dump);
		return 0;
	}
	/* VAD-gated TX (tx.c:234-245): superframe k is encoded only when
	 * gate[k] != 0; a gated-off superframe leaves the codec untouched and
	 * its 11 output bytes zero */
	if (!strcmp(argv[1], "encgate") && argc == 5) {
		long len, glen, k;
		int16_t *pcm = (int16_t *) read_file(argv[2], &len);
		unsigned char *gate = (unsigned char *) read_file(argv[3], &glen);
		unsigned char *bits = (unsigned char *) calloc(glen + 1, 11);
		short sp[BLOCK];
		FILE *f;
		melpe_i();
		for (k = 0; k < glen && (k + 1) * BLOCK * 2 <= len; k++) {
			if (!gate[k])
				continue;
			memcpy(sp, pcm + k * BLOCK, sizeof(sp));
			melpe_a(bits + k * 11, sp);
		}
		f = fopen(argv[4], "wb");
		fwrite(bits, 11, k, f);
		fclose(f);
		return 0;
	}
	if (!strcmp(argv[1], "dec") && (argc == 4 || argc == 5)) {
		long len, nsf;
		unsigned char *bits = (unsigned char *) read_file(argv[2], &len);
		int16_t *pcm;
		FILE *dump = argc == 5 ? fopen(argv[4], "wb") : NULL;
		FILE *f;
		nsf = len / 11;
		pcm = (int16_t *) calloc(nsf * BLOCK + 1, 2);
		decode_buffer(bits, nsf, pcm, dump);
		f = fopen(argv[3], "wb");
		fwrite(pcm, 2, nsf * BLOCK, f);
		fclose(f);
		if (dump)
			fclose(dump);
		return 0;
	}
	if (!strcmp(argv[1], "duplex") && argc == 6) {
		long plen, blen, k, nsf;
		int16_t *pcm = (int16_t *) read_file(argv[2], &plen);
		unsigned char *bits = (unsigned char *) read_file(argv[3], &blen);
		FILE *fb, *fp;
		int16_t out[BLOCK];
		unsigned char buf[11];
		nsf = plen / 2 / BLOCK;
		if (blen / 11 < nsf)
			nsf = blen / 11;
		fb = fopen(argv[4], "wb");
		fp = fopen(argv[5], "wb");
		melpe_i();
		for (k = 0; k < nsf; k++) {
			melpe_a(buf, pcm + k * BLOCK);
			fwrite(buf, 1, 11, fb);
			memcpy(buf, bits + k * 11, 11);
			melpe_s(out, buf);
			fwrite(out, 2, BLOCK, fp);
		}
		fclose(fb);
		fclose(fp);
		return 0;
	}
	if (!strcmp(argv[1], "npp") && argc == 4) {
		long len, k, nfr;
		/* read_file pads 4096 zero bytes: melpe_n's first call reads
		 * 256 samples (melpe/npp.c:178-179) */
		int16_t *pcm = (int16_t *) read_file(argv[2], &len);
		FILE *f;
		nfr = len / 2 / FRAME;
		melpe_i();
		for (k = 0; k < nfr; k++)
			melpe_n(pcm + k * FRAME);
		f = fopen(argv[3], "wb");
		fwrite(pcm, 2, nfr * FRAME, f);
		fclose(f);
		return 0;
	}
	if (!strcmp(argv[1], "encgen") && (argc == 7 || argc == 8)) {
		struct encgen_arg a;
		long nch = atol(argv[4]);
		a.seed = (uint32_t) strtoul(argv[2], 0, 0);
		a.ch0 = atol(argv[3]);
		a.nsf = atol(argv[5]);
		a.out_bits = argv[6];
		a.out_npp = argc == 8 ? argv[7] : NULL;
		make_file(a.out_bits, nch * a.nsf * 11);
		if (a.out_npp)
			make_file(a.out_npp, nch * a.nsf * BLOCK * 2);
		run_children(nch, encgen_one, &a);
		return 0;
	}
	if (!strcmp(argv[1], "decgen") && argc == 6) {
		struct decgen_arg a;
		long len, nch = atol(argv[3]);
		a.bits = (const unsigned char *) read_file(argv[2], &len);
		a.nsf = atol(argv[4]);
		a.out = argv[5];
		if (len < nch * a.nsf * 11) {
			fprintf(stderr, "short bitstream file\n");
			return 2;
		}
		make_file(a.out, nch * a.nsf * BLOCK * 2);
		run_children(nch, decgen_one, &a);
		return 0;
	}
	if (!strcmp(argv[1], "enc24gen") && (argc == 7 || argc == 8)) {
		struct encgen_arg a;
		long nch = atol(argv[4]);
		a.seed = (uint32_t) strtoul(argv[2], 0, 0);
		a.ch0 = atol(argv[3]);
		a.nsf = atol(argv[5]);
		a.out_bits = argv[6];
		a.out_npp = argc == 8 ? argv[7] : NULL;
		make_file(a.out_bits, nch * a.nsf * 7);
		if (a.out_npp)
			make_file(a.out_npp, nch * a.nsf * FRAME * 2);
		run_children(nch, enc24gen_one, &a);
		return 0;
	}
	if (!strcmp(argv[1], "dec24gen") && argc == 6) {
		struct decgen_arg a;
		long len, nch = atol(argv[3]);
		a.bits = (const unsigned char *) read_file(argv[2], &len);
		a.nsf = atol(argv[4]);
		a.out = argv[5];
		if (len < nch * a.nsf * 7) {
			fprintf(stderr, "short bitstream file\n");
			return 2;
		}
		make_file(a.out, nch * a.nsf * FRAME * 2);
		run_children(nch, dec24gen_one, &a);
		return 0;
	}
	fprintf(stderr, "bad command\n");
	return 1;
}
