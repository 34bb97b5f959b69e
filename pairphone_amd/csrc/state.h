/*
 * state.h -- explicit per-channel state of the engine.
 *
 * The reference keeps one codec instance per process in globals
 * (melpe/global.c:20-53) and ~90 function statics.
 * Here every one of them is a field of EncState / DecState, one instance per
 * channel in HBM; enc_reset()/dec_reset() give the state of a fresh process
 * (static initialisers + melp_ana_init / melp_syn_init, melpe/melpe.c:72-88).
 */
#ifndef MELPE_STATE_H
#define MELPE_STATE_H

#include "npp.h"

namespace mlp {

/* codec geometry (melpe/sc1200.h:60-140) */
#define FRAME 180
#define NF 3
#define BLOCK 540
#define LPC_ORD 10
#define NUM_HARM 10
#define NUM_BANDS 5
#define NUM_GAINFR 2
#define PITCHMIN 20
#define PITCHMAX 160
#define PITCHMIN_Q7 2560
#define PITCHMAX_Q7 20480
#define PITCH_FR 321
#define FRAME_BEG 70
#define FRAME_END 250
#define PITCH_BEG 90
#define IN_BEG 360
#define LPC_FRAME 200
#define LPF_ORD 6
#define DC_ORD 6
#define BPF_ORD 6
#define ENV_ORD 2
#define PIT_COR_LEN 220
#define PIT_SUBNUM 2
#define PIT_SUBFRAME 90
#define NODE 8
#define TRACK_NUM 9
#define CUR_TRACK 2
#define MAXPITCH 147
#define MINPITCH 20
#define MAX_LSF_STAGE 4
#define MSVQ_STAGES 4
#define SIG_LENGTH (LPF_ORD + PITCH_FR)
#define UV_PITCH_Q7 6400
#define DEFAULT_PITCH_Q7 6400
#define LOG_UV_PITCH_Q12 6963
#define MAX_JITTER_Q15 8192
#define BPTHRESH_Q14 9830
#define VJIT_Q14 8192
#define VMIN_Q14 13107
#define VOICED 0
#define UNVOICED 1
#define TRANSITION 0
#define SILENCE 3

struct MelpParam {	/* struct melp_param, melpe/sc1200.h:233 */
	int16_t pitch;	/* Q7 */
	int16_t lsf[LPC_ORD];	/* Q15 */
	int16_t gain[NUM_GAINFR];	/* Q8 */
	int16_t jitter;	/* Q15 */
	int16_t bpvc[NUM_BANDS];	/* Q14 */
	int16_t uv_flag;
	int16_t fs_mag[NUM_HARM];	/* Q13 */
};

struct QuantParam {	/* struct quant_param, melpe/sc1200.h:244 (no pointers) */
	int16_t pitch_index;
	int16_t lsf_index[NF][MAX_LSF_STAGE];
	int16_t gain_index[NUM_GAINFR];
	int16_t jit_index[NF];
	int16_t bpvc_index[NF];
	int16_t fs_index;
	int16_t uv_flag[NF];
	int16_t msvq_index[MSVQ_STAGES];
	int16_t fsvq_index;
};

struct ClassParam {	/* classParam, melpe/cprv.h:40 */
	int16_t classy, subEnergy, zeroCrosRate, peakiness, corx, pitch;
};

struct PitTrack {	/* pitTrackParam, melpe/cprv.h:34 */
	int16_t pit[NODE], weight[NODE], cost[NODE];
};

/* The analysis state is grouped by the task chain that owns it, each group
 * dword-aligned and contiguous, so the multi-wave analysis kernel
 * (ana_mw.h) can hand each group back to HBM from the wave that ran that
 * chain: the driver group (frames' pitch/gain chain, sc_ana, quantisers,
 * packing), classify's, pitchAuto's, and one per bandpass-voicing band. */

/* melpe/classify.c statics */
struct alignas(4) ClsState {
	int16_t cls_started;
	int16_t bpfdel[BPF_ORD + BPF_ORD / 3];
	int16_t back_sigbuf[PIT_COR_LEN - PIT_SUBFRAME];
};

/* melpe/pitch.c statics */
struct alignas(4) PautoState {
	int16_t pauto_started;
	int16_t lpbuf[PIT_COR_LEN], ivbuf[PIT_COR_LEN];
};

/* one band of melpe/melp_sub.c bpvc_ana's statics (:81-86 keep them as
 * [NUM_BANDS][..] arrays; here band-major) */
struct alignas(4) BandState {
	int16_t fsp[PITCH_FR - FRAME];	/* bpfsp[b] */
	int16_t delin[BPF_ORD], delout[BPF_ORD];	/* bpfdelin/out[b] */
	int16_t env[ENV_ORD], env2;	/* envdel[b], envdel2[b] */
};

/* The analysis state of one channel: everything analysis() reads or writes.
 * The lane kernels hold a private copy of this part only (not the NPP
 * state), and move just its live prefix, [0, ENC_ANA_LIVE): the other
 * chains' groups, the driver group and the carried speech history
 * hpspeech[0, IN_BEG).  What follows it -- the superframe's new samples
 * hpspeech[IN_BEG, IN_BEG + BLOCK) (dc_rmv writes each frame's before
 * melp_ana reads it) and sigbuf (each stage that uses it writes the part it
 * reads first) -- is per-superframe working storage, never read before it
 * is written; the host build (emu_encode_ana_split) fills it with a pattern
 * to check exactly that. */
struct alignas(16) EncAna {
	/* ---- the other chains' groups (ana_mw.h) ---- */
	ClsState cls;
	PautoState pa;
	BandState band[NUM_BANDS];	/* band[0] belongs to the driver group */
	/* ---- driver group ---- */
	/* melpe/global.c */
	int16_t dcdelin[DC_ORD], dcdelout_hi[DC_ORD], dcdelout_lo[DC_ORD];
	MelpParam par[NF];
	QuantParam qpar;
	int16_t voicedEn, silenceEn;
	int32_t voicedCnt;
	/* melpe/melp_ana.c */
	ClassParam classStat[TRACK_NUM];
	PitTrack pitTrack[TRACK_NUM];
	int16_t ana_started;
	int16_t lpfsp_delin[LPF_ORD], lpfsp_delout[LPF_ORD];
	int16_t pitch_avg, fpitch[2];
	int16_t sc_prev_sbp3, sc_prev_uv, sc_prev_pitch;
	/* melpe/melp_sub.c bpvc_ana's first-call flag */
	int16_t bp_started;
	/* melpe/pit_lib.c */
	int16_t pavg_started, good_pitch[NF];
	int16_t pana_started;
	int16_t lpres_delin[LPF_ORD], lpres_delout[LPF_ORD];
	int16_t pa_sigbuf[SIG_LENGTH];
	/* melpe/qnt12.c */
	int16_t pvq_prev_uv_flag, pvq_prev_pitch, pvq_prev_qpitch;
	int16_t lsf_started, qplsp[LPC_ORD];
	int16_t fsm_prev_uv, fsm_prev_fsmag[NUM_HARM];
	/* melpe/melp_chn.c */
	int16_t sync_bit;
	int16_t pad_;
	uint8_t chbuf[12];
	/* 2400 bps path: melpe/melp_ana.c top_lpc, melpe/melp_sub.c q_gain
	 * prev_gain */
	int16_t top_lpc[LPC_ORD];
	int16_t qg_prev_gain;
	int16_t pad24_;
	/* melpe/global.c speech history: [0, IN_BEG) carried, the rest the new
	 * superframe (working storage, see above); on a 16-byte boundary, so
	 * the live prefix ends on one (IN_BEG int16 = 45 x 16 bytes) */
	alignas(16) int16_t hpspeech[IN_BEG + BLOCK];
	/* melpe/melp_ana.c sigbuf: working storage */
	int16_t sigbuf[SIG_LENGTH];
};

/* the first byte of the driver group, the end of the live prefix */
#define ENC_DRV_BEG offsetof(EncAna, dcdelin)
#define ENC_ANA_LIVE (offsetof(EncAna, hpspeech) + sizeof(int16_t) * IN_BEG)
static_assert(ENC_ANA_LIVE % 16 == 0 && sizeof(EncAna) % 16 == 0,
	      "the lane kernels move the live prefix in 16-byte pieces (kern.h lane_copy_x4)");

struct EncState {
	NppState npp;
	EncAna a;	/* 16-byte aligned */
	uint32_t fmt_pad_[3];	/* the tag in the record's last 4 bytes (16-byte size) */
	/* record format tag (reset sets it, no kernel writes it):
	 * melpe_engine_import rejects records of another layout */
	uint32_t fmt;
};
static_assert(offsetof(EncState, fmt) + 4 == sizeof(EncState), "EncState's tag ends the record");
static_assert(offsetof(EncState, a) % 16 == 0 && sizeof(EncState) % 16 == 0, "16-byte record copies");

#define MIX_ORD 32
#define DISP_ORD 64

struct alignas(16) DecState {	/* 16-byte aligned: moved with dwordx4 (k_dec.hip) */
	/* ---- the excitation side: the channel read, the parameter
	 * interpolation and harm_syn_pitch (wave A of the two-wave decoder,
	 * decoder.h melp_syn_a) ---- */
	MelpParam par[NF];	/* melp_par: error paths read last superframe's */
	QuantParam qpar;	/* quant_par: ditto (uv_flag, indices) */
	/* melpe/melp_syn.c */
	MelpParam prev_par;
	int16_t syn_begin, erase;
	int16_t syn_started, noise_gain, prev_lpc_gain, prev_tilt;
	int16_t prev_pcof[MIX_ORD + 1], prev_ncof[MIX_ORD + 1];
	/* melpe/melp_chn.c low_rate_chn_read */
	int16_t rd_started, rd_prev_uv;
	int16_t rd_prev_fsmag[NUM_HARM], rd_qplsp[LPC_ORD];
	int16_t rd_prev_gain[2 * NF * NUM_GAINFR];
	uint8_t chbuf[12];
	/* melpe/dsp_sub.c rand_minstdgen */
	uint32_t seed;
	/* 2400 bps path: melpe/melp_sub.c q_gain_dec prev_gain, prev_gain_err */
	int16_t qgd_prev_gain, qgd_prev_err;
	/* ---- the filter side, from a 16-byte boundary to the end: the
	 * synthesis filters, scale_adj, the dispersion FIR, the postfilter
	 * (wave B, decoder.h melp_syn_b) ---- */
	/* melpe/melp_syn.c */
	alignas(16) int16_t sigsave[PITCHMAX];
	int16_t lpc_del[LPC_ORD], ase_del[LPC_ORD], tilt_del[1];
	int16_t disp_del[DISP_ORD];
	/* melpe/melp_sub.c scale_adj */
	int16_t prev_scale;
	/* melpe/postfilt.c */
	int16_t pf_hpm, pf_gain;
	int16_t pf_mem1[LPC_ORD], pf_mem2[LPC_ORD];
	int16_t pf_aFIR[LPC_ORD], pf_aIIR[LPC_ORD];
	int16_t hpf_din[2], hpf_dhi[2], hpf_dlo[2];
	int16_t lpf_din[2], lpf_dhi[2], lpf_dlo[2];
	uint32_t fmt_pad_;	/* the tag in the record's last 4 bytes (16-byte size) */
	uint32_t fmt;	/* record format tag, as EncState's */
};
/* the two sides' byte ranges of the record (the two-wave decoder writes each
 * back from the wave that owns it) */
#define DEC_B_BEG offsetof(DecState, sigsave)
static_assert(DEC_B_BEG % 16 == 0, "the filter side starts on a 16-byte boundary");
static_assert(offsetof(DecState, fmt) + 4 == sizeof(DecState), "DecState's tag ends the record");

/* Layout version of the records (bump on any change to EncState /
 * DecState); the tag also folds in the record size. */
#define MELPE_REC_LAYOUT 6u
#define ENC_REC_FMT (0x4d450000u ^ (MELPE_REC_LAYOUT << 24) ^ (uint32_t) sizeof(EncState))
#define DEC_REC_FMT (0x4d440000u ^ (MELPE_REC_LAYOUT << 24) ^ (uint32_t) sizeof(DecState))

/* melp_ana_init, melpe/melp_ana.c:475-506 (the part melpe_i re-runs) */
MD void enc_melpe_i(EncAna *e)
{
	for (int i = 0; i < IN_BEG + BLOCK; i++)
		e->hpspeech[i] = 0;
	for (int i = 0; i < TRACK_NUM; i++) {
		for (int k = 0; k < NODE; k++) {
			e->pitTrack[i].pit[k] = 50;
			e->pitTrack[i].weight[k] = SW_MAX_;
		}
		e->classStat[i].classy = UNVOICED;
		e->classStat[i].subEnergy = 5734;
		e->classStat[i].zeroCrosRate = 16384;
		e->classStat[i].peakiness = 2048;
		e->classStat[i].corx = 6554;
	}
}

/* fresh-process state: zero .bss, the reference's static initialisers, then
 * melpe_i() */
MD void enc_reset(EncState *e)
{
	int16_t *p = (int16_t *) e;
	for (unsigned i = 0; i < sizeof(EncState) / 2; i++)
		p[i] = 0;
	npp_reset(&e->npp);
	EncAna *a = &e->a;
	a->sc_prev_uv = UNVOICED;	/* melp_ana.c:525-527 */
	a->sc_prev_pitch = 6400;
	a->pvq_prev_uv_flag = 1;	/* qnt12.c:78-80 */
	a->pvq_prev_pitch = LOG_UV_PITCH_Q12;
	a->pvq_prev_qpitch = LOG_UV_PITCH_Q12;
	a->fsm_prev_uv = 1;	/* qnt12.c:1279 */
	enc_melpe_i(a);
	e->fmt = ENC_REC_FMT;
}

/* melp_syn_init, melpe/melp_syn.c:478-502 (the part melpe_i re-runs) */
MD void dec_melpe_i(DecState *d)
{
	d->prev_par.gain[0] = d->prev_par.gain[1] = 0;
	d->prev_par.pitch = UV_PITCH_Q7;
	Word16 t = 0;
	for (int i = 0; i < LPC_ORD; i++) {
		t = add(t, 2979);
		d->prev_par.lsf[i] = t;
	}
	d->prev_par.jitter = 0;
	for (int i = 0; i < NUM_BANDS; i++)
		d->prev_par.bpvc[i] = 0;
	d->syn_begin = 0;
	for (int i = 0; i < PITCHMAX; i++)
		d->sigsave[i] = 0;
	for (int i = 0; i < NUM_HARM; i++)
		d->prev_par.fs_mag[i] = 8192;
}

MD void dec_reset(DecState *d)
{
	int16_t *p = (int16_t *) d;
	for (unsigned i = 0; i < sizeof(DecState) / 2; i++)
		p[i] = 0;
	d->noise_gain = 2560;	/* melp_syn.c:165-166 */
	d->prev_lpc_gain = SW_MAX_;
	d->rd_prev_uv = 1;	/* melp_chn.c:460 */
	d->seed = 1;	/* dsp_sub.c:369 */
	dec_melpe_i(d);
	d->fmt = DEC_REC_FMT;
}

}  // namespace mlp

#endif
