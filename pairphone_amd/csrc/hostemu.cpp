/*
 * hostemu.cpp -- host build of the engine's DEVICE sources, for CPU-side
 * tests only (tests/test_hostemu.py).  It runs the very same per-channel
 * code that the HIP kernels run (ops.h .. codec headers compiled with g++
 * instead of hipcc), one channel after another, so the kernel logic can be
 * checked against the reference oracle in a container without a GPU.
 *
 * NOT part of the product: libmelpe_amd.so never loads it, and nothing in
 * pairphone_amd/ imports it.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "codec.h"
#if !defined(MELPE_OPCOUNT)	/* the census counts the reference's serial order */
#include "ana_mw.h"
#endif
#include "helpers_eval.h"
#include "codec2400.h"
#include "voice_crypt.h"
#include "vad.h"
#include "modem.h"

using namespace mlp;

struct emu_engine {
	int channels;
	std::vector<EncState> enc;
	std::vector<DecState> dec;
};

static NppScratch g_npp_scratch;

#if defined(MELPE_EXACT_STATS)
extern "C" { long melpe_exact_stats[6] = {0, 0, 0, 0, 0, 0}; }
#endif

#if defined(MELPE_OPCOUNT)
extern "C" {
uint64_t melpe_opcount[64];
uint64_t melpe_stagecount[64];
int melpe_opstage;
int melpe_opdepth;
}
#endif

extern "C" {

int emu_load_tables(const char *path)
{
	FILE *f = fopen(path, "rb");
	if (!f)
		return -1;
	size_t n = fread(g_tab, sizeof(int16_t), MELPE_TABLE_WORDS, f);
	fclose(f);
	if (n != MELPE_TABLE_WORDS)
		return -2;
	derive_all(&g_der);
	derive_lspgrid(g_der.lsp_cos, g_lspgrid);
	return 0;
}

emu_engine *emu_create(int channels)
{
	emu_engine *e = new emu_engine();
	e->channels = channels;
	e->enc.resize(channels);
	e->dec.resize(channels);
	for (int c = 0; c < channels; c++) {
		enc_reset(&e->enc[c]);
		dec_reset(&e->dec[c]);
	}
	return e;
}

void emu_destroy(emu_engine *e)
{
	delete e;
}

int emu_npp(emu_engine *e, int16_t *sp, int frames, int stride, int rate1200)
{
	for (int c = 0; c < e->channels; c++)
		for (int f = 0; f < frames; f++) {
			int16_t *x = sp + (size_t) c * stride + f * NPP_HOP;
			npp_frame(&e->enc[c].npp, &g_npp_scratch, x, x, rate1200 != 0);
		}
	return 0;
}

/* melpe_a on every channel: sp (C x 540) in/out, bits (C x 11) out */
int emu_encode(emu_engine *e, unsigned char *bits, int16_t *sp)
{
	for (int c = 0; c < e->channels; c++) {
		encode_superframe(&e->enc[c], &g_npp_scratch, sp + (size_t) c * BLOCK);
		for (int k = 0; k < 11; k++)
			bits[c * 11 + k] = e->enc[c].a.chbuf[k];
	}
	return 0;
}

/* the two halves of melpe_a, as the GPU runs them (k_enc_npp, k_enc_ana) */
int emu_encode_npp(emu_engine *e, int16_t *sp)
{
	for (int c = 0; c < e->channels; c++) {
		int16_t *x = sp + (size_t) c * BLOCK;
		for (int f = 0; f < NF; f++)
			npp_frame(&e->enc[c].npp, &g_npp_scratch, x + f * FRAME, x + f * FRAME);
	}
	return 0;
}

/* the split lane analysis as k_enc_ana / k_enc_harm / k_enc_tail run it,
 * with the Fourier magnitudes from the scalar find_harm on the written
 * residuals (the wave kernel's own arithmetic is checked on the GPU) */
int emu_encode_ana_split(emu_engine *e, unsigned char *bits, const int16_t *sp)
{
	static int16_t res[NF * LPC_FRAME];
	static EncAna L;	/* the lane's private copy (k_ana.hip AnaLane) */
	for (int c = 0; c < e->channels; c++) {
		EncAna *E = &L;
		for (int k = 0; k < NF * LPC_FRAME; k++)
			res[k] = (int16_t) 0x5a5a;	/* unvoiced rows stay unread */
		/* the live prefix in, the working storage a pattern (state.h):
		 * nothing may read it before writing it */
		memcpy(E, &e->enc[c].a, ENC_ANA_LIVE);
		memset((char *) E + ENC_ANA_LIVE, 0x5a + (c & 7), sizeof(EncAna) - ENC_ANA_LIVE);
		analysis_a(E, sp + (size_t) c * BLOCK, res);
		memcpy(&e->enc[c].a, E, ENC_ANA_LIVE);
		E = &e->enc[c].a;
		for (int i = 0; i < NF; i++) {
			MelpParam *par = &E->par[i];
			v_set(par->fs_mag, 8192, NUM_HARM);
			if (!par->uv_flag)
				find_harm(&res[i * LPC_FRAME], par->fs_mag, par->pitch, NUM_HARM, LPC_FRAME);
		}
		analysis_b(E);
		for (int k = 0; k < 11; k++)
			bits[c * 11 + k] = E->chbuf[k];
	}
	return 0;
}

int emu_encode_ana(emu_engine *e, unsigned char *bits, const int16_t *sp)
{
	for (int c = 0; c < e->channels; c++) {
		analysis(&e->enc[c].a, sp + (size_t) c * BLOCK);
		for (int k = 0; k < 11; k++)
			bits[c * 11 + k] = e->enc[c].a.chbuf[k];
	}
	return 0;
}

#if !defined(MELPE_OPCOUNT)
/* the multi-wave analysis (ana_mw.h) as k_enc_ana_mw runs it: nw physical
 * waves, each with its own private copy of the record, phase by phase (the
 * barriers), the exchange block and the HBM record the only shared data;
 * each wave writes back the state groups of its virtual waves */
struct HostXch {
	int16_t w[XS_WORDS];
	int16_t get(int k) const { return w[k]; }
	void put(int k, int16_t v) { w[k] = v; }
};

/* lsf_vq's per-channel score row (HBM on the GPU) */
struct HostDb {
	uint32_t v[LQ_ROW];
	uint32_t get(int u) const { return v[u]; }
	void put(int u, uint32_t x) { v[u] = x; }
};

int emu_encode_ana_mw(emu_engine *e, unsigned char *bits, const int16_t *sp, int nw)
{
	if (nw < 1 || nw > MW_NV)
		return -1;
	std::vector<EncAna> W(nw);
	for (int c = 0; c < e->channels; c++) {
		EncAna &rec = e->enc[c].a;
		const int16_t *x = sp + (size_t) c * BLOCK;
		HostXch xc;
		memset(&xc, 0x5a, sizeof xc);	/* nothing may read a slot before it is written */
		static HostDb db;
		memset(&db, 0xa5, sizeof db);
		AnaMwTmp tmp[MW_NV];
		for (int w = 0; w < nw; w++) {
			memset(&W[w], 0xa5 + w, sizeof(EncAna));	/* uncopied bytes: a pattern */
			ana_mw_copy_in(&W[w], &rec, w, nw);
			ana_mw_begin(&W[w], x);
		}
		for (int p = 0; p < MW_PHASES; p++)
			for (int w = 0; w < nw; w++)
				for (int v = w; v < MW_NV; v += nw)
					ana_mw_phase(&W[w], &rec, xc, db, tmp[v], v, p);
		for (int w = 0; w < nw; w++)
			for (int v = w; v < MW_NV; v += nw) {
				size_t off[2], len[2];
				int n = ana_mw_owned(v, off, len);
				for (int k = 0; k < n; k++)
					memcpy((char *) &rec + off[k], (const char *) &W[w] + off[k], len[k]);
			}
		for (int k = 0; k < 11; k++)
			bits[c * 11 + k] = rec.chbuf[k];
	}
	return 0;
}
#endif

/* host build of the helper self-test (helpers_eval.h), same layout as
 * melpe_helpers_eval_dev */
int emu_helpers_eval(int mode, const int16_t *src, const int32_t *args, int32_t *out, int n)
{
	for (int i = 0; i < n; i++) {
		alignas(4) int16_t buf[HE_N];
		memcpy(buf, src + (size_t) i * HE_N, sizeof buf);
		int32_t *o = out + (size_t) i * HE_OUT;
		memset(o, 0, sizeof(int32_t) * HE_OUT);
		he_eval(mode, buf, args[4 * i], args[4 * i + 1], args[4 * i + 2], o);
	}
	return 0;
}

/* melpe_s on every channel: bits (C x 11) in, sp (C x 540) out */
int emu_decode(emu_engine *e, int16_t *sp, const unsigned char *bits)
{
	for (int c = 0; c < e->channels; c++) {
		DecState *D = &e->dec[c];
		memcpy(D->chbuf, bits + c * 11, 11);
		decode_superframe(D, sp + (size_t) c * BLOCK);
	}
	return 0;
}

#if !defined(MELPE_OPCOUNT)
/* the two-wave decoder (decoder.h dec2_phase) as k_decode2 runs it: wave A
 * and wave B each on a private copy of the record, phase by phase, the two
 * hand-over buffers the only shared data; each writes back its own side */
struct HostHb {
	uint32_t *v;
	uint32_t get(int k) const { return v[k]; }
	void put(int k, uint32_t x) const { v[k] = x; }
};

int emu_decode2(emu_engine *e, int16_t *sp, const unsigned char *bits)
{
	static uint32_t hb[2][HB_WORDS];
	static DecState W[2];
	for (int c = 0; c < e->channels; c++) {
		DecState *D = &e->dec[c];
		memset(hb, 0x5a, sizeof hb);	/* nothing may read a word before it is written */
		for (int r = 0; r < 2; r++)
			W[r] = *D;
		memcpy(W[0].chbuf, bits + c * 11, 11);
		memset(W[1].chbuf, 0xa5, 11);	/* B never reads the channel */
		int16_t *out = sp + (size_t) c * BLOCK;
		for (int p = 0; p < DEC2_PHASES; p++)
			for (int r = 0; r < 2; r++)
				dec2_phase(&W[r], out, HostHb{hb[0]}, HostHb{hb[1]}, r, p);
		memcpy(D, &W[0], DEC_B_BEG);
		memcpy((char *) D + DEC_B_BEG, (const char *) &W[1] + DEC_B_BEG, sizeof(DecState) - DEC_B_BEG);
	}
	return 0;
}
#endif

/* per-superframe debug view of channel c: melp_par (3 x 30 int16) and
 * quant_par (30 int16), in the layout oracle/ref_tool.c dumps */
int emu_enc_params(emu_engine *e, int c, int16_t *out)
{
	const EncAna *E = &e->enc[c].a;
	memcpy(out, E->par, sizeof(E->par));
	const QuantParam *q = &E->qpar;
	int16_t *w = out + 90;
	int k = 0;
	w[k++] = q->pitch_index;
	for (int i = 0; i < NF; i++)
		for (int j = 0; j < MAX_LSF_STAGE; j++)
			w[k++] = q->lsf_index[i][j];
	for (int i = 0; i < NUM_GAINFR; i++)
		w[k++] = q->gain_index[i];
	for (int i = 0; i < NF; i++)
		w[k++] = q->jit_index[i];
	for (int i = 0; i < NF; i++)
		w[k++] = q->bpvc_index[i];
	w[k++] = q->fs_index;
	for (int i = 0; i < NF; i++)
		w[k++] = q->uv_flag[i];
	for (int i = 0; i < MSVQ_STAGES; i++)
		w[k++] = q->msvq_index[i];
	w[k++] = q->fsvq_index;
	return k;
}

/* the single-stream engine's melp_par / quant_par / chbuf hand-over around
 * melpe_s (engine.hip k_share_params), channel 0 */
int emu_share(emu_engine *e, int dir)
{
	EncAna *E = &e->enc[0].a;
	DecState *D = &e->dec[0];
	if (dir == 0) {
		memcpy(D->par, E->par, sizeof(D->par));
		D->qpar = E->qpar;
	} else {
		memcpy(E->par, D->par, sizeof(E->par));
		E->qpar = D->qpar;
		memcpy(E->chbuf, D->chbuf, 11);
	}
	return 0;
}

/* decoder's melp_par of channel c after the last superframe (3 x 30 int16) */
int emu_dec_params(emu_engine *e, int c, int16_t *out)
{
	memcpy(out, e->dec[c].par, sizeof(e->dec[c].par));
	return 90;
}

/* basic-op census (count build only): copies and clears the counters;
 * returns the number of ops, or -1 in a normal build */
int emu_opcount(uint64_t *out, int n)
{
#if defined(MELPE_OPCOUNT)
	for (int i = 0; i < n && i < 64; i++) {
		out[i] = melpe_opcount[i];
		melpe_opcount[i] = 0;
	}
	return 37;
#else
	(void) out;
	(void) n;
	return -1;
#endif
}

/* per-stage census (count build only): ops attributed to the innermost
 * PROF_SCOPE stage (index k+1; 0 = outside any stage); copies and clears */
int emu_stagecount(uint64_t *out, int n)
{
#if defined(MELPE_OPCOUNT)
	for (int i = 0; i < n && i < 64; i++) {
		out[i] = melpe_stagecount[i];
		melpe_stagecount[i] = 0;
	}
	return 64;
#else
	(void) out;
	(void) n;
	return -1;
#endif
}

const char *emu_op_names(void)
{
	return MELPE_OP_NAMES;
}


/* host build of the voice-frame crypt (voice_crypt.h), same layout as
 * melpe_voice_crypt_host */
int emu_voice_crypt(unsigned char *pkts, const uint32_t *counters, const unsigned char *keys,
		    const uint8_t *invert, int channels, int packets, int dir)
{
	for (int c = 0; c < channels; c++) {
		uint32_t key[4];
		memcpy(key, keys + 16 * (size_t) c, 16);
		for (int k = 0; k < packets; k++)
			vc_apply(pkts + ((size_t) c * packets + k) * VC_PKT_BYTES,
				 counters[c] + (uint32_t) k, key, dir, invert ? invert[c] : 0);
	}
	return 0;
}

#if defined(MELPE_OPCOUNT)
uint64_t melpe_vad_ops;
int melpe_vad_depth;
#endif

/* VAD basic-op census since the last call (count build only; else 0) */
uint64_t emu_vad_opcount(void)
{
#if defined(MELPE_OPCOUNT)
	uint64_t n = melpe_vad_ops;
	melpe_vad_ops = 0;
	return n;
#else
	return 0;
#endif
}

int emu_vad_state_bytes(void)
{
	return (int) sizeof(VadState);
}

/* host build of k_vad: `nsf` superframes of C channels, sp C x (nsf*540),
 * votes C x nsf, state C records (zeroed by the caller = vad2_reset) */
int emu_vad(unsigned char *state, const int16_t *sp, uint8_t *votes, int channels, int nsf)
{
	VadState *st = (VadState *) state;
	for (int c = 0; c < channels; c++)
		for (int k = 0; k < nsf; k++)
			votes[(size_t) c * nsf + k] = (uint8_t) va_superframe(
				sp + ((size_t) c * nsf + k) * 540, &st[c]);
	return 0;
}

/* 2400 bps mode (codec2400.h): sp C x 180 in/out (NPP at RATE2400, then
 * analysis), bits C x 7 out; decode bits C x 7 -> sp C x 180 */
int emu_encode2400(emu_engine *e, unsigned char *bits, int16_t *sp)
{
	for (int c = 0; c < e->channels; c++) {
		EncState *S = &e->enc[c];
		int16_t *x = sp + (size_t) c * FRAME;
		npp_frame(&S->npp, &g_npp_scratch, x, x, false);
		analysis24(&S->a, x);
		memcpy(bits + (size_t) c * R24_BYTES, S->a.chbuf, R24_BYTES);
	}
	return 0;
}

int emu_decode2400(emu_engine *e, int16_t *sp, const unsigned char *bits)
{
	for (int c = 0; c < e->channels; c++) {
		DecState *D = &e->dec[c];
		memcpy(D->chbuf, bits + (size_t) c * R24_BYTES, R24_BYTES);
		decode_frame24(D, sp + (size_t) c * FRAME);
	}
	return 0;
}

/* raw state records (test diagnostics): which 1 = EncState, 2 = DecState */
long emu_state_bytes(int which)
{
	return which == 1 ? (long) sizeof(EncState) : (long) sizeof(DecState);
}

int emu_export(emu_engine *e, int which, int c, void *out)
{
	if (which == 1)
		memcpy(out, &e->enc[c], sizeof(EncState));
	else
		memcpy(out, &e->dec[c], sizeof(DecState));
	return 0;
}

/* host build of the modem (modem.h) */
int emu_modem_state_bytes(void)
{
	return (int) sizeof(ModemState);
}

void emu_modem_reset(unsigned char *state, int channels)
{
	for (int c = 0; c < channels; c++)
		modem_reset((ModemState *) state + c);
}

/* pkts C x K x 11 -> pcm C x K x 3240 */
int emu_modulate(unsigned char *state, const uint8_t *pkts, int16_t *pcm, int channels, int packets)
{
	for (int c = 0; c < channels; c++) {
		ModemState *S = (ModemState *) state + c;
		for (int k = 0; k < packets; k++) {
			const uint8_t *d = pkts + ((size_t) c * packets + k) * 11;
			int16_t *o = pcm + ((size_t) c * packets + k) * MODEM_PKT_SAMPLES;
			int prev = S->lastb;
			for (int t = 0; t < MODEM_BITS; t++) {
				int b = modem_tx_bit(d, t);
				for (int ii = 0; ii < 36; ii++)
					o[t * 36 + ii] = modem_sample(b, prev, S->vadtr, ii);
				prev = b;
			}
			S->lastb = prev;
			S->vadtr ^= 1;
		}
	}
	return 0;
}

/* `calls` Demodulate calls per channel on pcm C x stride from pos[c];
 * data C x 12 in/out, out C x calls x 12, ret C x calls */
int emu_demodulate(unsigned char *state, const int16_t *pcm, long stride, int32_t *pos,
		   uint8_t *data, uint8_t *out, int32_t *ret, int channels, int calls)
{
	for (int c = 0; c < channels; c++) {
		ModemState *S = (ModemState *) state + c;
		for (int k = 0; k < calls; k++) {
			int32_t r = -1;
			if (pos[c] >= 0 && pos[c] + MODEM_LOOKAHEAD <= stride) {
				r = modem_demod(S, pcm + (size_t) c * stride + pos[c], data + 12 * (size_t) c);
				pos[c] += r;
			}
			for (int i = 0; i < 12; i++)
				out[((size_t) c * calls + k) * 12 + i] = data[12 * (size_t) c + i];
			ret[(size_t) c * calls + k] = r;
			if (r < 0)
				break;
		}
	}
	return 0;
}

}  // extern "C"
