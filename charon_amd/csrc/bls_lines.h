// Miller-loop line precomputation for a G2 point.
//
// The optimal-ate loop over |x| = 0xd201000000010000 evaluates 68 lines
// (63 tangents + 5 chords).  They depend only on the G2 argument, so they are
// computed once per point and stored: for the signature side the G1 argument
// is the fixed -g1 and is folded in; for H(m) the lines are stored with the
// G1 factor left out (l1', l4') and evaluated per public key as
// l1 = l1' * (-x_pk), l4 = l4' * y_pk.  H(m) is shared by the n partials of a
// DV, so its lines are computed once per message.
#pragma once
#include "bls_pairing.h"

namespace tbg {

constexpr int N_LINES = 68;
constexpr int LINE_WORDS = 3 * 2 * NL;               // (l0, l1, l4) in Fp2
constexpr int LINES_WORDS = N_LINES * LINE_WORDS;    // per G2 point: 5712 words

TBG_HD void line_store(uint32_t* dst, const Line& l) {
  const Fp* f[6] = {&l.l0.c0, &l.l0.c1, &l.l1.c0, &l.l1.c1, &l.l4.c0, &l.l4.c1};
  for (int k = 0; k < 6; ++k)
    for (int i = 0; i < NL; ++i) dst[k * NL + i] = f[k]->l[i];
}

TBG_HD Line line_load(const uint32_t* src) {
  Line l;
  Fp* f[6] = {&l.l0.c0, &l.l0.c1, &l.l1.c0, &l.l1.c1, &l.l4.c0, &l.l4.c1};
  for (int k = 0; k < 6; ++k)
    for (int i = 0; i < NL; ++i) f[k]->l[i] = src[k * NL + i];
  return l;
}

// All 68 lines of Q in loop order; nxP / yP = (-x_P, y_P) to fold P in, or
// (1, 1) (Montgomery one) to leave it out.  INL = true inlines the doubling
// and addition steps (kernel callers only: the loop body is ~100 KB).
template <bool INL>
TBG_HD void g2_lines_t(const G2A& Q, const Fp& nxP, const Fp& yP, uint32_t* out) {
  G2J T = jac_from_aff(Q);
  int idx = 0;
  for (int i = 62; i >= 0; --i) {
    line_store(out + LINE_WORDS * idx++, INL ? miller_dbl_in(T, nxP, yP) : miller_dbl(T, nxP, yP));
    if ((X_ABS >> i) & 1) line_store(out + LINE_WORDS * idx++, miller_add(T, Q, nxP, yP));
  }
}
TBG_NI void g2_lines(const G2A& Q, const Fp& nxP, const Fp& yP, uint32_t* out) { g2_lines_t<false>(Q, nxP, yP, out); }

}  // namespace tbg
