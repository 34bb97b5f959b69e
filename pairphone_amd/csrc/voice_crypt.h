/*
 * voice_crypt.h -- PairPhone's voice-frame encryption,
 * the step right after melpe_a on the TX side (tx.c:269 -> crp.c:819) and
 * right before melpe_s on the RX side (rx.c:340-358 -> crp.c:980).
 *
 * Reference (crp.c:986-1027, VoiceEnc / VoiceDec):
 *   gamma = first 11 bytes squeezed from the Keccak sponge
 *           (r = 576, c = 1024, crypto/Keccak512_data.h:28-30) after
 *           absorbing counter (4 bytes little-endian, crp.c:322-327) || key
 *           (16 bytes: skey[0..15] to encrypt, skey[16..31] to decrypt);
 *   gamma[10] &= 1 (81 bits); pkt[i] ^= gamma[i], i < 11.
 *   VoiceDec first inverts the packet when the channel polarity flag is
 *   negative (crp.c:1011-1015): pkt[0..9] ^= 0xFF, pkt[10] ^= 1.
 *
 * The 20 absorbed bytes fit in one 72-byte block, so the sponge is one
 * Keccak-f[1600] on a fixed-shape padded block: Sponge_init (no key, no
 * header: crypto/sponge.c:268-271) zeroes the state, Sponge_data SP_NORMAL
 * (:311-409) XORs the 20 bytes into bytes 0..19 without permuting, and
 * Sponge_finalize (:415-432) XORs 0x01 at byte 20 and 0x80 at byte 71,
 * permutes once and copies the first bytes out.  The permutation is the
 * standard Keccak-f[1600] (crypto/sponge.c:205-264: theta, rho+pi through
 * KeccakF_PiLane / KeccakF_RotationConstants, chi, iota; 24 rounds).
 *
 * Here the state is 25 64-bit lanes in registers and every round is fully
 * unrolled, so all lane indices and rotations are compile-time constants.
 * Shared by the GPU kernel (engine.hip) and the host-emulation build.
 */
#ifndef MELPE_VOICE_CRYPT_H
#define MELPE_VOICE_CRYPT_H

#include <stdint.h>

#ifndef MELPE_HD
#if defined(__HIPCC__)
#define MELPE_HD __host__ __device__
#else
#define MELPE_HD
#endif
#endif

#define VC_PKT_BYTES 11
#define VC_KEY_BYTES 16

static MELPE_HD inline uint64_t vc_rol(uint64_t a, int n)
{
	return n ? (a << n) | (a >> (64 - n)) : a;
}

/* Keccak-f[1600] in place, A[x + 5y] */
static MELPE_HD inline void vc_keccak_f(uint64_t A[25])
{
	const uint64_t RC[24] = {
		0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL,
		0x8000000080008000ULL, 0x000000000000808bULL, 0x0000000080000001ULL,
		0x8000000080008081ULL, 0x8000000000008009ULL, 0x000000000000008aULL,
		0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
		0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL,
		0x8000000000008003ULL, 0x8000000000008002ULL, 0x8000000000000080ULL,
		0x000000000000800aULL, 0x800000008000000aULL, 0x8000000080008081ULL,
		0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
	/* rho offset of lane x + 5y */
	const int R[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
			   25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
#pragma unroll
	for (int r = 0; r < 24; r++) {
		uint64_t C[5], B[25];
#pragma unroll
		for (int x = 0; x < 5; x++)
			C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
#pragma unroll
		for (int x = 0; x < 5; x++) {
			uint64_t d = C[(x + 4) % 5] ^ vc_rol(C[(x + 1) % 5], 1);
#pragma unroll
			for (int y = 0; y < 25; y += 5)
				A[y + x] ^= d;
		}
		/* rho + pi: B[y, 2x + 3y] = rot(A[x, y]) */
#pragma unroll
		for (int x = 0; x < 5; x++)
#pragma unroll
			for (int y = 0; y < 5; y++)
				B[y + 5 * ((2 * x + 3 * y) % 5)] = vc_rol(A[x + 5 * y], R[x + 5 * y]);
		/* chi */
#pragma unroll
		for (int y = 0; y < 25; y += 5)
#pragma unroll
			for (int x = 0; x < 5; x++)
				A[y + x] = B[y + x] ^ (~B[y + (x + 1) % 5] & B[y + (x + 2) % 5]);
		A[0] ^= RC[r];
	}
}

/* gamma = H(counter LE || key)[0..10], with gamma[10] &= 1, returned as
 * lo = bytes 0..7, hi = bytes 8..10 (little-endian) */
static MELPE_HD inline void vc_gamma(uint32_t counter, const uint32_t key[4], uint64_t *lo,
				     uint64_t *hi)
{
	uint64_t A[25];
#pragma unroll
	for (int i = 0; i < 25; i++)
		A[i] = 0;
	A[0] = (uint64_t) counter | ((uint64_t) key[0] << 32);		/* bytes 0..7 */
	A[1] = (uint64_t) key[1] | ((uint64_t) key[2] << 32);		/* bytes 8..15 */
	A[2] = (uint64_t) key[3] | ((uint64_t) 0x01 << 32);		/* bytes 16..19, pad at 20 */
	A[8] = (uint64_t) 0x80 << 56;					/* pad at byte 71 */
	vc_keccak_f(A);
	*lo = A[0];
	*hi = A[1] & 0x1FFFFULL;	/* bytes 8, 9 and bit 0 of byte 10 */
}

/* VoiceEnc (dir 0) / VoiceDec (dir 1) on one 11-byte packet */
static MELPE_HD inline void vc_apply(unsigned char *pkt, uint32_t counter, const uint32_t key[4],
				     int dir, int invert)
{
	uint64_t lo, hi;
	vc_gamma(counter, key, &lo, &hi);
	if (dir && invert) {
		lo = ~lo;
		hi ^= 0x1FFFFULL;	/* bytes 8, 9 ^= 0xFF; byte 10 ^= 1 */
	}
#pragma unroll
	for (int i = 0; i < 8; i++)
		pkt[i] ^= (unsigned char) (lo >> (8 * i));
#pragma unroll
	for (int i = 0; i < 3; i++)
		pkt[8 + i] ^= (unsigned char) (hi >> (8 * i));
}

#endif
