// Test harness: the device line parser (csrc/textparse_line.h, the body of
// k_parse) compiled for the CPU, so tests/test_textparse.py can check its
// decisions against the Python host parser without a GPU.  Test
// infrastructure only: nothing in the product loads this library.
#include "../../ruleset-analysis_amd/csrc/textparse_line.h"

// text: 4-byte aligned, readable up to a multiple of 4 bytes past off[n];
// word = 1 parses through the word-cached accessor (the device's LDS path),
// 0 through byte loads (its fallback path).
extern "C" void parse_lines_host(const uint8_t* text, const uint64_t* off, uint64_t n, const rsa_parse_ifc* ifcs,
                                 uint32_t n_ifcs, const rsa_parse_spell* spells, uint32_t n_spells,
                                 rsa_tuple* tuples, uint32_t* ts, uint32_t* disp, int word) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = off[i], b = off[i + 1];
    uint64_t len = b - a;
    if (len && text[b - 1] == '\n') --len;
    if (word == 2) {   // the direct-HBM accessor (k_parse<..., true>)
      const rsa_text::GWordLn s{reinterpret_cast<const uint32_t*>(text), text, a, off[n], (uint32_t)len, ~0ull, 0u};
      rsa_text::parse_line(s, ifcs, n_ifcs, spells, n_spells, tuples[i], ts[i], disp[i]);
    } else if (word) {
      const rsa_text::WordLn s{reinterpret_cast<const uint32_t*>(text), (uint32_t)a, (uint32_t)len};
      rsa_text::parse_line(s, ifcs, n_ifcs, spells, n_spells, tuples[i], ts[i], disp[i]);
    } else {
      const rsa_text::ByteLn s{text + a, (uint32_t)len};
      rsa_text::parse_line(s, ifcs, n_ifcs, spells, n_spells, tuples[i], ts[i], disp[i]);
    }
  }
}

// The reducer drop-in's per-line parse (textparse.hip k_parse<true>): each
// line's fields and the same-key flag against the previous line.
extern "C" void reduce_lines_host(const uint8_t* text, const uint64_t* off, uint64_t n, const rsa_parse_spell* spells,
                                  uint32_t n_spells, rsa_tuple* tuples, uint32_t* ts, uint32_t* disp, int word) {
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = off[i], b = off[i + 1];
    uint64_t len = b - a;
    if (len && text[b - 1] == '\n') --len;
    const rsa_text::ByteLn s{text + a, (uint32_t)len};
    if (word == 2) {
      const rsa_text::GWordLn w{reinterpret_cast<const uint32_t*>(text), text, a, off[n], (uint32_t)len, ~0ull, 0u};
      rsa_text::reduce_line(w, spells, n_spells, tuples[i], ts[i], disp[i]);
    } else if (word) {
      const rsa_text::WordLn w{reinterpret_cast<const uint32_t*>(text), (uint32_t)a, (uint32_t)len};
      rsa_text::reduce_line(w, spells, n_spells, tuples[i], ts[i], disp[i]);
    } else {
      rsa_text::reduce_line(s, spells, n_spells, tuples[i], ts[i], disp[i]);
    }
    if (i > 0 && disp[i] != RSA_RED_NOISE) {
      const uint64_t pa = off[i - 1];
      uint64_t plen = a - pa;
      if (plen && text[a - 1] == '\n') --plen;
      if (rsa_text::same_key(s, rsa_text::ByteLn{text + pa, (uint32_t)plen})) disp[i] |= RSA_RED_SAME_KEY;
    }
  }
}

// The template fast path against the general one: for every line gb_match
// accepts, out[i] = 0 (not the template), 1 (template; built_template's
// groups and hit flag equal built_search's and hit_test's), 2 (template, but
// they differ -- a bug).
extern "C" void template_check_host(const uint8_t* text, const uint64_t* off, uint64_t n, uint8_t* out) {
  using namespace rsa_text;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = off[i], b = off[i + 1];
    uint64_t len = b - a;
    if (len && text[b - 1] == '\n') --len;
    const ByteLn s{text + a, (uint32_t)len};
    Mapped m;
    Hdr h;
    Reduced r, g;
    bool hit = false;
    out[i] = 0;
    if (!gb_match(s, m, h) || !built_template(s, m, h, r, hit)) continue;
    const bool ok = built_search(s, g) && hit == hit_test(s);
    const Span* x[8] = {&r.time, &r.mon, &r.day, &r.year, &r.word, &r.for_ip, &r.to_ip, &r.to_port};
    const Span* y[8] = {&g.time, &g.mon, &g.day, &g.year, &g.word, &g.for_ip, &g.to_ip, &g.to_port};
    bool same = ok;
    for (int k = 0; k < 8 && same; ++k) same = x[k]->a == y[k]->a && x[k]->b == y[k]->b;
    out[i] = same ? 1 : 2;
  }
}

// The template scan (k_parse's pass) against the general parse: per line
// out[i] = 0 (not accepted: the slow pass decides), 1 (accepted, same
// disposition / tuple / timestamp code as parse_line), 2 (accepted but
// different -- a bug).
// word = 1: tpl_finish reads through the LDS-staged word accessor (the buffer
// must stay readable 20 bytes past off[n]), 0: byte reads.
extern "C" void tpl_check_host(const uint8_t* text, const uint64_t* off, uint64_t n, const rsa_parse_ifc* ifcs,
                               uint32_t n_ifcs, const rsa_parse_spell* spells, uint32_t n_spells, uint8_t* out,
                               int word) {
  using namespace rsa_text;
  uint32_t slot[tpl::kSlotWords];
  static constexpr tpl::ClsTable kCls = tpl::cls_table();
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = off[i], b = off[i + 1];
    uint64_t len = b - a;
    if (len && text[b - 1] == '\n') --len;
    const ByteLn s{text + a, (uint32_t)len};
    rsa_tuple t1, t2;
    uint32_t ts1 = 0, ts2 = 0, d1 = 0, d2 = 0;
    out[i] = 0;
    if (!tpl::scan(s, tpl::kProg, kCls.t, slot)) continue;
    const WordLn w{reinterpret_cast<const uint32_t*>(text), (uint32_t)a, (uint32_t)len};
    if (!(word ? tpl_finish(w, slot, ifcs, n_ifcs, spells, n_spells, t1, ts1, d1)
               : tpl_finish(s, slot, ifcs, n_ifcs, spells, n_spells, t1, ts1, d1)))
      continue;
    parse_line(s, ifcs, n_ifcs, spells, n_spells, t2, ts2, d2);
    const bool same = d1 == d2 && ts1 == ts2 && t1.src == t2.src && t1.dst == t2.dst && t1.sport == t2.sport &&
                      t1.dport == t2.dport && t1.list == t2.list && t1.flags == t2.flags && t1.pspell == t2.pspell;
    out[i] = same ? 1 : 2;
  }
}
