// textparse_line.h — the per-line parse of textparse.hip (k_parse), as
// __host__ __device__ code so that tests can also run it on the CPU
// (tests/native/textparse_host.cpp) against the Python host parser.
#ifndef RSA_TEXTPARSE_LINE_H
#define RSA_TEXTPARSE_LINE_H

#include <stdint.h>

#include "../../include/ruleset_hip.h"

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace rsa_text {

#define RSA_HD __host__ __device__ __forceinline__

// One lane per line, bytes read through the line accessor.
// Line accessors: s[i] = byte i of the line, s.n = its length without '\n'.
struct ByteLn {              // plain byte loads (any buffer)
  const uint8_t* p;
  uint32_t n;
  RSA_HD uint32_t operator[](uint32_t i) const { return p[i]; }
};
struct WordLn {              // one 4-byte load per byte read (LDS staging): no per-lane word cache, whose
  const uint32_t* w32;       // compare-and-branch cost more than the extra LDS reads (8 % on k_parse,
  uint32_t o;                // profiles/r03l_text_8M_*.json); buffer readable up to the line's last word;
  uint32_t n;                // o = byte offset of the line in it
  RSA_HD uint32_t operator[](uint32_t i) const {
    const uint32_t pos = o + i;
    return (w32[pos >> 2] >> ((pos & 3u) * 8u)) & 0xFFu;
  }
};

struct GWordLn {             // global 4-byte loads with a one-word cache (no staging); bytes of the
  const uint32_t* w32;       // buffer's last, partial word are read one by one
  const uint8_t* b8;         // the same buffer, as bytes
  uint64_t o;                // byte offset of the line
  uint64_t nb;               // bytes in the buffer
  uint32_t n;
  mutable uint64_t ci;
  mutable uint32_t cw;
  RSA_HD uint32_t operator[](uint32_t i) const {
    const uint64_t pos = o + i, wi = pos >> 2;
    if (wi != ci) {
      ci = wi;
      if (4 * wi + 4 <= nb) {
        cw = w32[wi];
      } else {
        cw = 0;
        for (uint32_t k = 0; k < 4; ++k)
          if (4 * wi + k < nb) cw |= (uint32_t)b8[4 * wi + k] << (8 * k);
      }
    }
    return (cw >> ((uint32_t)(pos & 3u) * 8u)) & 0xFFu;
  }
};

struct GWordU {              // global 4-byte loads, one per byte read, no per-lane branch: the word of
  const uint32_t* w32;       // the buffer's last, partial bytes comes from `tail`
  uint64_t o;                // byte offset of the line
  uint64_t nw;               // whole words in the buffer
  uint32_t tail;             // the partial last word (zero padded)
  uint32_t n;
  RSA_HD uint32_t operator[](uint32_t i) const {
    const uint64_t pos = o + i, wi = pos >> 2;
    const uint32_t w = wi < nw ? w32[wi] : tail;
    return (w >> ((uint32_t)(pos & 3u) * 8u)) & 0xFFu;
  }
};

RSA_HD bool is_dig(uint32_t c) { return c - '0' < 10u; }
RSA_HD bool is_upper(uint32_t c) { return c - 'A' < 26u; }
RSA_HD bool is_lower(uint32_t c) { return c - 'a' < 26u; }
RSA_HD bool is_alpha(uint32_t c) { return (c | 32u) - 'a' < 26u; }
RSA_HD bool is_ifc(uint32_t c) { return is_alpha(c) || is_dig(c) || c == '_' || c == '-'; }
RSA_HD bool is_ipch(uint32_t c) { return is_dig(c) || c == '.'; }
RSA_HD bool is_tsch(uint32_t c) { return is_dig(c) || c == ':'; }

enum Cls { kDig, kAlpha, kIfc, kIp, kTs };
template <int C>
RSA_HD bool in_cls(uint32_t c) {
  return C == kDig ? is_dig(c) : C == kAlpha ? is_alpha(c) : C == kIfc ? is_ifc(c) : C == kIp ? is_ipch(c) : is_tsch(c);
}
// end of the run of class C starting at p
template <int C, class S>
RSA_HD uint32_t run(const S& s, uint32_t p) {
  while (p < s.n && in_cls<C>(s[p])) ++p;
  return p;
}
// s[p ..] starts with the literal
template <class S, int N>
RSA_HD bool lit(const S& s, uint32_t p, const char (&w)[N]) {
  if (p + (N - 1) > s.n) return false;
#pragma unroll
  for (int i = 0; i < N - 1; ++i)
    if (s[p + i] != (uint8_t)w[i]) return false;
  return true;
}
// largest k in [lo, hi] where the literal starts, or -1
template <class S, int N>
RSA_HD int64_t last_lit(const S& s, int64_t lo, int64_t hi, const char (&w)[N]) {
  if (hi > (int64_t)s.n - (N - 1)) hi = (int64_t)s.n - (N - 1);
  for (int64_t k = hi; k >= lo; --k)
    if (lit(s, (uint32_t)k, w)) return k;
  return -1;
}
// \d\d:\d\d:\d\d
template <class S>
RSA_HD bool hms(const S& s, uint32_t p) {
  return p + 8 <= s.n && is_dig(s[p]) && is_dig(s[p + 1]) && s[p + 2] == ':' && is_dig(s[p + 3]) &&
         is_dig(s[p + 4]) && s[p + 5] == ':' && is_dig(s[p + 6]) && is_dig(s[p + 7]);
}

struct Span {
  uint32_t a, b;
};

struct Mapped {             // get_builtconn's fields
  bool inbound, udp;
  Span if1, ip1, p1, if2, ip2, p2;
  Span par1;                // the text of the first \([^)]*\)
  uint32_t tag_d, proto;    // positions of the severity digit and of TCP/UDP
};

// Where gb_match found the header (parse_line's template fast path).
struct Hdr {
  uint32_t hms1, m2, d2a, d2b, ya, q, k;   // k: the '%' whose rest matched
  bool single, opt;                        // single spaces after both months; device date present
};

// The rest of logparse._GB after `.*?`, at the '%' + 1 position p.
template <class S>
RSA_HD bool gb_rest(const S& s, uint32_t p, Mapped& m) {
  if (lit(s, p, "ASA")) p += 3;
  else if (lit(s, p, "FWSM")) p += 4;
  else if (lit(s, p, "PIX")) p += 3;
  else return false;
  if (p + 3 > s.n || s[p] != '-' || !is_dig(s[p + 1]) || s[p + 2] != '-') return false;
  m.tag_d = p + 1;
  p += 3;
  if (p + 6 > s.n) return false;
  for (int i = 0; i < 6; ++i)
    if (!is_dig(s[p + i])) return false;
  p += 6;
  if (!lit(s, p, ": Built ")) return false;
  p += 8;
  if (lit(s, p, "inbound ")) {
    m.inbound = true;
    p += 8;
  } else if (lit(s, p, "outbound ")) {
    m.inbound = false;
    p += 9;
  } else {
    return false;
  }
  if (lit(s, p, "TCP")) m.udp = false;
  else if (lit(s, p, "UDP")) m.udp = true;
  else return false;
  m.proto = p;
  p += 3;
  if (!lit(s, p, " connection ")) return false;
  p += 12;
  uint32_t e = run<kDig>(s, p);
  if (e == p || e >= s.n || s[e] != ' ') return false;
  p = e + 1;
  if (!lit(s, p, "for ")) return false;
  p += 4;
  e = run<kIfc>(s, p);
  if (e == p || e >= s.n || s[e] != ':') return false;
  m.if1 = {p, e};
  p = e + 1;
  e = run<kIp>(s, p);
  if (e == p || e >= s.n || s[e] != '/') return false;
  m.ip1 = {p, e};
  p = e + 1;
  e = run<kDig>(s, p);
  if (e == p || !lit(s, e, " (")) return false;
  m.p1 = {p, e};
  p = e + 2;
  m.par1.a = p;
  while (p < s.n && s[p] != ')') ++p;   // [^)]*
  if (p >= s.n) return false;
  m.par1.b = p;
  ++p;
  if (!lit(s, p, " to ")) return false;
  p += 4;
  e = run<kIfc>(s, p);
  if (e == p || e >= s.n || s[e] != ':') return false;
  m.if2 = {p, e};
  p = e + 1;
  e = run<kIp>(s, p);
  if (e == p || e >= s.n || s[e] != '/') return false;
  m.ip2 = {p, e};
  p = e + 1;
  e = run<kDig>(s, p);
  if (e == p) return false;
  m.p2 = {p, e};
  return true;
}

// logparse._GB.match(line): header, optional device date, lazy .*? over the
// '%' positions (the first one whose rest matches wins).  The optional group
// is taken when it matches: skipping it cannot change the outcome, since its
// text holds no '%'.
template <class S>
RSA_HD bool gb_match(const S& s, Mapped& m, Hdr& h) {
  if (s.n < 3 || !is_upper(s[0]) || !is_lower(s[1]) || !is_lower(s[2])) return false;
  uint32_t p = 3;
  if (p >= s.n || s[p] != ' ') return false;
  while (p < s.n && s[p] == ' ') ++p;
  h.single = p == 4;
  uint32_t e = run<kDig>(s, p);
  if (e - p < 1 || e - p > 2 || e >= s.n || s[e] != ' ') return false;
  p = e + 1;
  if (!hms(s, p) || p + 8 >= s.n || s[p + 8] != ' ') return false;
  h.hms1 = p;
  p += 9;
  uint32_t q = p;
  h.opt = false;
  {
    uint32_t t = p;
    if (t + 3 <= s.n && is_upper(s[t]) && is_lower(s[t + 1]) && is_lower(s[t + 2]) && t + 3 < s.n && s[t + 3] == ' ') {
      h.m2 = t;
      t += 3;
      while (t < s.n && s[t] == ' ') ++t;
      h.single = h.single && t == h.m2 + 4;
      e = run<kDig>(s, t);
      if (e - t >= 1 && e - t <= 2 && e < s.n && s[e] == ' ') {
        h.d2a = t;
        h.d2b = e;
        t = e + 1;
        e = run<kDig>(s, t);
        if (e - t == 4 && e < s.n && s[e] == ' ') {
          h.ya = t;
          t = e + 1;
          if (hms(s, t) && t + 10 <= s.n && s[t + 8] == ':' && s[t + 9] == ' ') {
            q = t + 10;
            h.opt = true;
          }
        }
      }
    }
  }
  h.q = q;
  for (uint32_t k = q; k < s.n; ++k)
    if (s[k] == '%' && gb_rest(s, k + 1, m)) {
      h.k = k;
      return true;
    }
  return false;
}

template <class S>
RSA_HD bool gb_match(const S& s, Mapped& m) {
  Hdr h;
  return gb_match(s, m, h);
}

struct Reduced {            // connlist-reducer.py:25 BUILT captures used downstream
  Span time, mon, day, year, word, for_ip, to_ip, to_port;
};

// After `[a-zA-Z]+ [0-9 ]?[0-9] `: groups 1-4, then the three greedy `.*`
// (candidates tried from the last occurrence down, nested as the engine does).
template <class S>
RSA_HD bool built_tail(const S& s, uint32_t p, Reduced& r) {
  uint32_t e = run<kTs>(s, p);
  if (e == p || e >= s.n || s[e] != ' ') return false;
  r.time = {p, e};
  p = e + 1;
  e = run<kAlpha>(s, p);
  if (e == p || e >= s.n || s[e] != ' ') return false;
  r.mon = {p, e};
  p = e + 1;
  e = run<kDig>(s, p);
  if (e == p || e >= s.n || s[e] != ' ') return false;
  r.day = {p, e};
  p = e + 1;
  e = run<kDig>(s, p);
  if (e == p || e >= s.n || s[e] != ' ') return false;
  r.year = {p, e};
  p = e + 1;
  for (int64_t k1 = last_lit(s, p, (int64_t)s.n, " Built "); k1 >= (int64_t)p;
       k1 = last_lit(s, p, k1 - 1, " Built ")) {
    uint32_t t = (uint32_t)k1 + 7;
    if (lit(s, t, "out")) t += 3;
    else if (lit(s, t, "in")) t += 2;
    else continue;
    if (!lit(s, t, "bound ")) continue;
    t += 6;
    e = run<kAlpha>(s, t);
    if (e == t || e >= s.n || s[e] != ' ') continue;
    r.word = {t, e};
    const uint32_t q2 = e + 1;
    for (int64_t k2 = last_lit(s, q2, (int64_t)s.n, " for "); k2 >= (int64_t)q2;
         k2 = last_lit(s, q2, k2 - 1, " for ")) {
      uint32_t u = (uint32_t)k2 + 5;
      e = run<kIfc>(s, u);
      if (e == u || e >= s.n || s[e] != ':') continue;
      u = e + 1;
      e = run<kIp>(s, u);
      if (e == u || e >= s.n || s[e] != '/') continue;
      r.for_ip = {u, e};
      u = e + 1;
      e = run<kDig>(s, u);
      if (e == u || e >= s.n || s[e] != ' ') continue;
      const uint32_t q3 = e + 1;
      for (int64_t k3 = last_lit(s, q3, (int64_t)s.n, " to "); k3 >= (int64_t)q3;
           k3 = last_lit(s, q3, k3 - 1, " to ")) {
        uint32_t v = (uint32_t)k3 + 4;
        e = run<kIfc>(s, v);
        if (e == v || e >= s.n || s[e] != ':') continue;
        v = e + 1;
        e = run<kIp>(s, v);
        if (e == v || e >= s.n || s[e] != '/') continue;
        r.to_ip = {v, e};
        v = e + 1;
        e = run<kDig>(s, v);
        if (e == v) continue;
        r.to_port = {v, e};
        return true;
      }
    }
  }
  return false;
}

// BUILT.search(line): leftmost start.  A start inside a letter run has the
// same continuation as the run's first letter, so only run starts are tried;
// `[0-9 ]?` is tried taken, then skipped.
template <class S>
RSA_HD bool built_search(const S& s, Reduced& r) {
  for (uint32_t s0 = 0; s0 < s.n; ++s0) {
    if (!is_alpha(s[s0])) continue;
    const uint32_t e = run<kAlpha>(s, s0);
    const uint32_t p = e + 1;
    if (e < s.n && s[e] == ' ') {
      if (p + 2 < s.n && (is_dig(s[p]) || s[p] == ' ') && is_dig(s[p + 1]) && s[p + 2] == ' ' &&
          built_tail(s, p + 3, r))
        return true;
      if (p + 1 < s.n && is_dig(s[p]) && s[p + 1] == ' ' && built_tail(s, p + 2, r)) return true;
    }
    s0 = e;   // the next start is past this run (the loop's ++ skips the non-letter at e)
  }
  return false;
}

template <class S>
RSA_HD bool hit_test(const S& s) {   // '-6-302013' / '-6-302015' anywhere (connlist-reducer.py:146)
  if (s.n < 9) return false;
  for (uint32_t k = 0; k + 9 <= s.n; ++k)
    if (s[k] == '-' && s[k + 1] == '6' && lit(s, k + 2, "-30201") && (s[k + 8] == '3' || s[k + 8] == '5')) return true;
  return false;
}

template <class S>
RSA_HD bool span_eq(const S& s, Span x, Span y) {
  if (x.b - x.a != y.b - y.a) return false;
  for (uint32_t i = 0; i < x.b - x.a; ++i)
    if (s[x.a + i] != s[y.a + i]) return false;
  return true;
}

// canonical dotted quad (what str(IP) prints back) -> value
template <class S>
RSA_HD bool ipv4_canon(const S& s, Span x, uint32_t& v) {
  uint32_t p = x.a, val = 0;
  for (int o = 0; o < 4; ++o) {
    const uint32_t e = run<kDig>(s, p);
    if (e > x.b || e == p || e - p > 3 || (e - p > 1 && s[p] == '0')) return false;
    uint32_t octet = 0;
    for (uint32_t i = p; i < e; ++i) octet = octet * 10 + (s[i] - '0');
    if (octet > 255) return false;
    val = val << 8 | octet;
    if (o < 3) {
      if (e >= x.b || s[e] != '.') return false;
      p = e + 1;
    } else if (e != x.b) {
      return false;
    }
  }
  v = val;
  return true;
}

// int(text) of a digit run, saturating above 65535 (the caller defers those)
template <class S>
RSA_HD uint32_t port_val(const S& s, Span x) {
  uint32_t v = 0;
  for (uint32_t i = x.a; i < x.b; ++i) {
    v = v * 10 + (s[i] - '0');
    if (v > 65535u) return 65536u;
  }
  return v;
}

template <class S>
RSA_HD bool port_canon(const S& s, Span x) { return x.b - x.a == 1 || s[x.a] != '0'; }

template <class S>
RSA_HD uint32_t small_num(const S& s, Span x) {   // <= 4 digits
  uint32_t v = 0;
  for (uint32_t i = x.a; i < x.b; ++i) v = v * 10 + (s[i] - '0');
  return v;
}

// connlist-reducer.py:163-165 as a code: year(4 digits, 2000..2127)-MM-DD
// (day zfill(2) <= 31) HH:MM:SS (h < 24, m, s < 60); false = not codable
template <class S>
RSA_HD bool ts_code(const S& s, const Reduced& r, uint32_t& code) {
  const char* const months = "JanFebMarAprMayJunJulAugSepOctNovDec";
  if (r.mon.b - r.mon.a != 3) return false;
  int mo = -1;
  for (int k = 0; k < 12; ++k)
    if (s[r.mon.a] == (uint8_t)months[3 * k] && s[r.mon.a + 1] == (uint8_t)months[3 * k + 1] &&
        s[r.mon.a + 2] == (uint8_t)months[3 * k + 2]) {
      mo = k;
      break;
    }
  if (mo < 0) return false;
  if (r.year.b - r.year.a != 4 || r.day.b - r.day.a > 2 || r.time.b - r.time.a != 8) return false;
  const uint32_t y = small_num(s, r.year), d = small_num(s, r.day);
  if (y < RSA_TS_YEAR0 || y >= RSA_TS_YEAR0 + 128 || d > 31) return false;
  const uint32_t t = r.time.a;
  if (!hms(s, t)) return false;
  const uint32_t hh = (s[t] - '0') * 10 + (s[t + 1] - '0'), mm = (s[t + 3] - '0') * 10 + (s[t + 4] - '0'),
                 ss = (s[t + 6] - '0') * 10 + (s[t + 7] - '0');
  if (hh > 23 || mm > 59 || ss > 59) return false;
  code = ((((y - RSA_TS_YEAR0) * 12u + (uint32_t)mo) * 32u + d) * 86400u) + hh * 3600u + mm * 60u + ss;
  return true;
}

RSA_HD bool is_parch(uint32_t c) { return is_dig(c) || c == '.' || c == '/'; }

template <class S>
RSA_HD bool no_dash(const S& s, Span x) {
  for (uint32_t i = x.a; i < x.b; ++i)
    if (s[i] == '-') return false;
  return true;
}

// The template fast path of parse_line.  A line of exactly the form
//   Mmm D HH:MM:SS Mmm D YYYY HH:MM:SS: %TAG-d-dddddd: Built DIR PROTO
//   connection N for IF:IP/P (IP/P) to IF:IP/P (IP/P)
// (single spaces; D one or two digits; the parenthesised texts [0-9./]*; the
// line ends at the last ')') has one ' Built ', one ' for ' and one ' to '
// after the device date, so connlist-reducer.py:25's BUILT.search matches at
// the line's start with groups (HH:MM:SS of the syslog header, the device
// date's month, day and year, PROTO, the first IP, the second IP and P) --
// what built_search returns after its backtracking, read off gb_match's
// positions instead.  The hit test needs no scan either when no interface
// name holds a '-': the only '-' are then the tag's.  False: not the
// template, the general path decides.
template <bool kScan = true, class S>
RSA_HD bool built_template(const S& s, const Mapped& m, const Hdr& h, Reduced& r, bool& hit) {
  if (!h.opt || !h.single || h.k != h.q) return false;
  for (uint32_t i = m.par1.a; i < m.par1.b; ++i)
    if (!is_parch(s[i])) return false;
  uint32_t p = m.p2.b;
  if (!lit(s, p, " (")) return false;
  p += 2;
  while (p < s.n && is_parch(s[p])) ++p;
  if (p + 1 != s.n || s[p] != ')') return false;
  r.time = {h.hms1, h.hms1 + 8};
  r.mon = {h.m2, h.m2 + 3};
  r.day = {h.d2a, h.d2b};
  r.year = {h.ya, h.ya + 4};
  r.word = {m.proto, m.proto + 3};
  r.for_ip = m.ip1;
  r.to_ip = m.ip2;
  r.to_port = m.p2;
  if (no_dash(s, m.if1) && no_dash(s, m.if2)) {
    const uint32_t t = m.tag_d;
    hit = s[t] == '6' && lit(s, t + 2, "30201") && (s[t + 7] == '3' || s[t + 7] == '5');
  } else {
    if constexpr (!kScan) return false;   // (kScan false: no scanning code in the caller's kernel)
    hit = hit_test(s);
  }
  return true;
}

// Disposition of a line the template pass left to the general one (k_parse
// with kDefer; never leaves the library).
constexpr uint32_t kLineDefer = 0xFEu;

// The whole line: disposition (RSA_LINE_* | interface << 8), tuple, timestamp
// code.  kDefer: a classified line outside the template form is not parsed
// further (disposition kLineDefer): the general path, whose backtracking
// searches cost a whole wave for one such lane, runs on those lines alone.
template <bool kDefer = false, class S>
RSA_HD void parse_line(const S& s, const rsa_parse_ifc* ifcs, uint32_t n_ifcs, const rsa_parse_spell* spells,
                       uint32_t n_spells, rsa_tuple& tup_out, uint32_t& ts_out, uint32_t& d_out) {
  rsa_tuple tup = {0u, 0u, 0, 0, 0, 0, 0};
  uint32_t ts = 0, d = RSA_LINE_IGNORE;
#if defined(RSA_TP_PROF) && RSA_TP_PROF == 1   // timing experiment: no parse
  tup.src = s.n;
  tup_out = tup;
  ts_out = ts;
  d_out = d;
  return;
#endif
  {
    Mapped m;
    Hdr h;
#if defined(RSA_TP_PROF) && RSA_TP_PROF >= 2   // timing experiment: the mapper regex (+ template) only
    {
      const bool g = gb_match(s, m, h);
      Reduced r;
      bool hit = false;
      const bool f = RSA_TP_PROF == 3 && g && built_template(s, m, h, r, hit);
      tup.src = g ? m.ip1.b + m.p2.b : 0u;
      tup.dst = f ? r.year.a + r.time.b + hit : 0u;
      tup_out = tup;
      ts_out = ts;
      d_out = d;
      return;
    }
#endif
    if (gb_match(s, m, h)) {
      d = RSA_LINE_CLASSIFY;
      const Span src = m.inbound ? m.ip1 : m.ip2, dst = m.inbound ? m.ip2 : m.ip1;
      const Span sp = m.inbound ? m.p1 : m.p2, dp = m.inbound ? m.p2 : m.p1;
      const Span ifc = m.inbound ? m.if1 : m.if2;
      uint32_t vs = 0, vd = 0;
      const uint32_t ps = port_val(s, sp), pd = port_val(s, dp);
      // FirewallRule._address validation of the text (mapper.py:138-142): the
      // device takes canonical dotted quads only
      if (!ipv4_canon(s, src, vs) || !ipv4_canon(s, dst, vd)) d = RSA_LINE_HOST;
      int32_t found = -1;
      const uint32_t il = ifc.b - ifc.a;
      if (d == RSA_LINE_CLASSIFY) {
        if (il > RSA_IFC_NAME_MAX) {
          d = RSA_LINE_HOST;
        } else {
          for (uint32_t k = 0; k < n_ifcs && found < 0; ++k) {
            if (ifcs[k].len != il) continue;
            bool eq = true;
            for (uint32_t c = 0; c < il && eq; ++c) eq = s[ifc.a + c] == (uint8_t)ifcs[k].name[c];
            if (eq) found = (int32_t)k;
          }
          if (found < 0) {
            d = RSA_LINE_NOACL;
          } else if (ifcs[found].kind == RSA_LINE_MISSING) {
            d = RSA_LINE_MISSING | ((uint32_t)found << 8);
          } else if (ifcs[found].kind != RSA_LINE_CLASSIFY) {
            d = RSA_LINE_HOST;
          }
        }
      }
      if (d == RSA_LINE_CLASSIFY) {
        const uint32_t lid = m.udp ? ifcs[found].list_udp : ifcs[found].list_tcp;
        if (lid == RSA_LIST_HOST || ps > 65535u || pd > 65535u) d = RSA_LINE_HOST;
        tup.src = vs;
        tup.dst = vd;
        tup.sport = (uint16_t)ps;
        tup.dport = (uint16_t)pd;
        tup.list = (uint16_t)lid;
        uint32_t flags = RSA_F_VALID;
        Reduced r;
        bool hit = false;
        const bool fast = built_template<!kDefer>(s, m, h, r, hit);
        bool built = fast;
        if constexpr (kDefer) {
          // the general searches are not even compiled into the template
          // pass (code size: the kernel stays in the instruction cache)
          if (!fast && d == RSA_LINE_CLASSIFY) {
            tup_out = rsa_tuple{0u, 0u, 0, 0, 0, 0, 0};
            ts_out = 0;
            d_out = kLineDefer;
            return;
          }
        } else {
          if (!fast) {
            hit = hit_test(s);
            built = d == RSA_LINE_CLASSIFY && built_search(s, r);
          }
        }
        if (hit) flags |= RSA_F_HIT;
        if (d == RSA_LINE_CLASSIFY && built) {
          flags |= RSA_F_BUILT;
          uint32_t vf = 0, vt = 0;
          if (span_eq(s, r.for_ip, src) && span_eq(s, r.to_ip, dst) && span_eq(s, r.to_port, dp)) {
          } else if (span_eq(s, r.for_ip, dst) && span_eq(s, r.to_ip, src) && span_eq(s, r.to_port, sp)) {
            flags |= RSA_F_SWAP;
          } else {
            d = RSA_LINE_HOST;
          }
          if (!ipv4_canon(s, r.for_ip, vf) || !ipv4_canon(s, r.to_ip, vt) || !port_canon(s, r.to_port))
            d = RSA_LINE_HOST;
          if (hit && !ts_code(s, r, ts)) d = RSA_LINE_HOST;
          int32_t sid = -1;
          const uint32_t wl = r.word.b - r.word.a;
          for (uint32_t k = 0; k < n_spells && sid < 0; ++k) {
            if (spells[k].len != wl) continue;
            bool eq = true;
            for (uint32_t c = 0; c < wl && eq; ++c) eq = s[r.word.a + c] == (uint8_t)spells[k].word[c];
            if (eq) sid = (int32_t)k;
          }
          if (sid < 0) d = RSA_LINE_HOST;
          else tup.pspell = (uint8_t)sid;
        }
        tup.flags = (uint8_t)flags;
      }
      if (d != RSA_LINE_CLASSIFY) {
        tup = rsa_tuple{0u, 0u, 0, 0, 0, 0, 0};
        ts = 0;
      }
    }
  }
  tup_out = tup;
  ts_out = ts;
  d_out = d;
}

// ---- The template pass as one position-synchronous scan (k_parse).
//
// parse_line's sequential form runs data-dependent loops per lane (runs of
// digits, literals, searches): a wave pays for every loop of every lane, and
// the exec-mask bookkeeping of that divergence is scalar work the CU's one
// scalar unit serialises over its four SIMDs (~16K SALU per 64-line wave).
// Here every lane steps through its line one byte per iteration, all lanes on
// the same byte index, through a fixed program of segments (literal bytes, or
// runs of a character class with length bounds, each followed by one literal
// byte), with branch-free updates of running values: the decimal value of the
// current digit group, the dotted-quad value, the last eight letters, the run
// start, and at each run end the field's value into a per-lane slot.  Only
// the canonical form is accepted (exactly built_template's lines, plus the
// device's canonical-text conditions); anything else is left to the general
// parse.  Every accepted line gets parse_line's own disposition, tuple and
// timestamp code (tests/test_textparse.py checks that on the CPU).
namespace tpl {

enum Field : uint32_t {
  fM1, fHH, fMM, fSS, fM2, fD2, fY, fTAG, fSEV, fMSG, fDIR, fPROTO, fIF1, fIP1, fP1, fIF2, fIP2, fP2, kFields,
  fNone = 31
};
// character classes
constexpr uint32_t cD = 1, cU = 2, cL = 4, cDot = 8, cSl = 16, cDash = 32, cUnd = 64;
constexpr uint32_t cls_of(uint32_t c) {
  return (c - '0' < 10u ? cD : 0u) | (c - 'A' < 26u ? cU : 0u) | (c - 'a' < 26u ? cL : 0u) | (c == '.' ? cDot : 0u) |
         (c == '/' ? cSl : 0u) | (c == '-' ? cDash : 0u) | (c == '_' ? cUnd : 0u);
}

// segment: literal / follow byte 8 | class mask 8 (0: a literal) | min 3 | max 8 | field 5
constexpr uint32_t R(uint32_t msk, uint32_t mn, uint32_t mx, char follow, uint32_t fld) {
  return (uint32_t)(uint8_t)follow | msk << 8 | mn << 16 | mx << 19 | fld << 27;
}
constexpr uint32_t L(char ch) { return (uint32_t)(uint8_t)ch | (uint32_t)fNone << 27; }
constexpr uint32_t kEndSeg = 7u << 16 | (uint32_t)fNone << 27;   // a literal that matches nothing
constexpr uint32_t cIfc = cD | cU | cL | cDash | cUnd;

// Mmm D HH:MM:SS Mmm D YYYY HH:MM:SS: %TAG-d-dddddd: Built DIR PROTO connection N
// for IF:IP/P (IP/P) to IF:IP/P (IP/P)
constexpr uint32_t kProg[] = {
    R(cU | cL, 3, 3, ' ', fM1), R(cD, 1, 2, ' ', fNone), R(cD, 2, 2, ':', fHH), R(cD, 2, 2, ':', fMM),
    R(cD, 2, 2, ' ', fSS), R(cU | cL, 3, 3, ' ', fM2), R(cD, 1, 2, ' ', fD2), R(cD, 4, 4, ' ', fY),
    R(cD, 2, 2, ':', fNone), R(cD, 2, 2, ':', fNone), R(cD, 2, 2, ':', fNone), L(' '), L('%'),
    R(cU, 3, 4, '-', fTAG), R(cD, 1, 1, '-', fSEV), R(cD, 6, 6, ':', fMSG), L(' '), L('B'), L('u'), L('i'), L('l'),
    L('t'), L(' '), R(cL, 7, 8, ' ', fDIR), R(cU, 3, 3, ' ', fPROTO), L('c'), L('o'), L('n'), L('n'), L('e'),
    L('c'), L('t'), L('i'), L('o'), L('n'), L(' '), R(cD, 1, 255, ' ', fNone), L('f'), L('o'), L('r'), L(' '),
    R(cIfc, 1, 255, ':', fIF1), R(cD | cDot, 1, 255, '/', fIP1), R(cD, 1, 255, ' ', fP1), L('('),
    R(cD | cDot | cSl, 0, 255, ')', fNone), L(' '), L('t'), L('o'), L(' '), R(cIfc, 1, 255, ':', fIF2),
    R(cD | cDot, 1, 255, '/', fIP2), R(cD, 1, 255, ' ', fP2), L('('), R(cD | cDot | cSl, 0, 255, ')', fNone),
    kEndSeg};
constexpr uint32_t kProgLen = sizeof(kProg) / sizeof(kProg[0]);
constexpr uint32_t kSlotWords = kFields + 1;   // one span per field + a dummy slot

constexpr uint32_t pack3(char a, char b, char c) { return (uint32_t)(uint8_t)a << 16 | (uint32_t)(uint8_t)b << 8 | (uint8_t)c; }

// One byte of the scan: byte c at index i of the line.  P: the program (LDS
// copy on the device), C: the class of each byte value (cls_of, an LDS table
// on the device), Q: the lane's kSlotWords slot words, each field's span as
// start | length << 16.  act 0 (the line already ended): no state changes,
// the slot write goes to the dummy slot.  The conditions are 0/1 integers
// combined with integer ops and bit selects (v_bfi): booleans would live in
// scalar lane masks, and their and/or/select bookkeeping is scalar work that
// the CU's one scalar unit serialises over its four SIMDs.
// The descriptor prog[seg] is read on every byte: carrying the next ones in
// registers (no LDS read on the byte-to-byte chain) measured slower on gfx950
// (16M-line text job: parse 6.41 vs 6.08 ms, profiles/r04w_text16_*.json).
struct State {
  uint32_t seg = 0, cnt = 0, pos0 = 0, ok = 1;
};
template <class P>
RSA_HD State start(P) {
  return State{};
}
RSA_HD uint32_t lt01(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a - b) >> 63); }   // a < b
RSA_HD uint32_t nz01(uint32_t a) { return a ? 1u : 0u; }
RSA_HD uint32_t sel(uint32_t m01, uint32_t a, uint32_t b) {   // m01 ? a : b, as a bit select
  const uint32_t m = 0u - m01;
  return (a & m) | (b & ~m);
}
template <class P, class C, class Q>
RSA_HD void step(State& st, uint32_t i, uint32_t c, uint32_t act, P prog, C cls, Q slot) {
  const uint32_t desc = prog[st.seg];
  const uint32_t lit = desc & 0xFFu, msk = (desc >> 8) & 0xFFu, mn = (desc >> 16) & 7u, mx = (desc >> 19) & 0xFFu,
                 fld = desc >> 27;
  const uint32_t is_run = nz01(msk);
  const uint32_t cnt = st.cnt;
  st.pos0 = sel(1u - nz01(cnt), i, st.pos0);
  const uint32_t cont = nz01((uint32_t)cls[c] & msk) & lt01(cnt, mx);   // (msk 0: a literal, never a run byte)
  const uint32_t rend = act & st.ok & is_run & (cont ^ 1u);              // a run ends here: its span into the slot
  slot[sel(rend & lt01(fld, kFields), fld, kFields)] = st.pos0 | cnt << 16;
  const uint32_t step_ok = cont | (((lt01(cnt, mn) ^ 1u) | (is_run ^ 1u)) & (1u - nz01(c ^ lit)) &
                                   nz01(desc ^ kEndSeg));
  const uint32_t nok = st.ok & step_ok;
  const uint32_t adv = act & nok & (cont ^ 1u) & lt01(st.seg + 1, kProgLen);
  st.seg += adv;
  st.ok = sel(act, nok, st.ok);
  st.cnt = sel(act, (cnt + 1) & (0u - cont), cnt);
}

// The scan of a whole line.  True: the line has the template form.  All
// lanes step together (the loop runs to the longest line of the wave).
template <class S, class P, class C, class Q>
RSA_HD bool scan(const S& s, P prog, C cls, Q slot) {
  if (s.n > 0xFFFFu) return false;
  State st = start(prog);
  for (uint32_t i = 0; i < s.n; ++i) step(st, i, s[i], 1u, prog, cls, slot);
  return st.ok && prog[st.seg] == kEndSeg;
}

// the byte classes as a table (the device copies it to LDS)
struct ClsTable {
  uint8_t t[256];
};
constexpr ClsTable cls_table() {
  ClsTable x{};
  for (uint32_t c = 0; c < 256; ++c) x.t[c] = (uint8_t)cls_of(c);
  return x;
}

}  // namespace tpl

// ---- 16 bytes of a line in registers (tpl_finish).  Each field is read as
// one block (a few independent word loads, all issued before any test) and
// decoded with selects, instead of one dependent byte load per step of a
// per-field loop.  Bytes past the line are unspecified: callers mask by the
// field's length.
struct B16 {
  uint32_t w[4];
  RSA_HD uint32_t b(uint32_t i) const { return (w[i >> 2] >> (8u * (i & 3u))) & 0xFFu; }   // i static
};
RSA_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t r) {   // (hi:lo) >> r, r < 32
  return r ? (lo >> r) | (hi << (32u - r)) : lo;
}
RSA_HD B16 funnel5(const uint32_t (&x)[5], uint32_t r) {
  return B16{{funnel(x[1], x[0], r), funnel(x[2], x[1], r), funnel(x[3], x[2], r), funnel(x[4], x[3], r)}};
}
template <class S>
RSA_HD B16 bytes16(const S& s, uint32_t p) {   // any accessor: byte reads, zero past the line
  B16 r{{0u, 0u, 0u, 0u}};
  for (uint32_t i = 0; i < 16; ++i)
    if (p + i < s.n) r.w[i >> 2] |= (uint32_t)s[p + i] << (8u * (i & 3u));
  return r;
}
// LDS-staged words: the buffer must stay readable 20 bytes past the line
RSA_HD B16 bytes16(const WordLn& s, uint32_t p) {
  const uint32_t pos = s.o + p, q = pos >> 2;
  const uint32_t x[5] = {s.w32[q], s.w32[q + 1], s.w32[q + 2], s.w32[q + 3], s.w32[q + 4]};
  return funnel5(x, (pos & 3u) * 8u);
}
RSA_HD B16 bytes16(const GWordU& s, uint32_t p) {
  const uint64_t pos = s.o + p, q = pos >> 2;
  uint32_t x[5];
  for (uint32_t k = 0; k < 5; ++k) x[k] = q + k < s.nw ? s.w32[q + k] : (q + k == s.nw ? s.tail : 0u);
  return funnel5(x, (uint32_t)(pos & 3u) * 8u);
}
// bytes [0, n) of a block as a little-endian mask per word
RSA_HD uint32_t lmask(uint32_t word, uint32_t n) {
  const uint32_t lo = 4u * word;
  return n >= lo + 4 ? 0xFFFFFFFFu : (n <= lo ? 0u : (1u << (8u * (n - lo))) - 1u);
}
RSA_HD bool b16_eq(const B16& x, const B16& y, uint32_t n) {   // first n (<= 16) bytes equal
  uint32_t d = 0;
  for (uint32_t k = 0; k < 4; ++k) d |= (x.w[k] ^ y.w[k]) & lmask(k, n);
  return d == 0;
}
RSA_HD bool b16_has(const B16& x, uint32_t n, uint32_t c) {   // byte c among the first n
  uint32_t hit = 0;
  for (uint32_t i = 0; i < 16; ++i) hit |= (uint32_t)(i < n) & (uint32_t)(x.b(i) == c);
  return hit != 0;
}
// decimal value of the digits [o, o + n) of a block (n <= N, the text is digits)
template <uint32_t N>
RSA_HD uint32_t b16_num(const B16& x, uint32_t o, uint32_t n) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < N; ++i) {
    const uint32_t c = x.b(o + i) - '0';
    v = i < n ? v * 10u + c : v;
  }
  return v;
}
// port_val of a digit field: saturating at 65536 (fields past 16 bytes: 65536, the general parse decides)
RSA_HD uint32_t b16_port(const B16& x, uint32_t n) {
  uint32_t v = n > 16u ? 65536u : 0u;
  for (uint32_t i = 0; i < 16; ++i) {
    const uint32_t t = v * 10u + (x.b(i) - '0');
    v = (i < n && v < 65536u) ? (t > 65535u ? 65536u : t) : v;
  }
  return v;
}
RSA_HD B16 b16_shr(const B16& x, uint32_t nb) {   // drop the first nb (< 4) bytes
  const uint32_t r = 8u * nb;
  return B16{{funnel(x.w[1], x.w[0], r), funnel(x.w[2], x.w[1], r), funnel(x.w[3], x.w[2], r), funnel(0u, x.w[3], r)}};
}
// ipv4_canon over a block: d{1,3}(.d{1,3}){3}, no leading zeros, octets <= 255
RSA_HD bool b16_ipv4(const B16& x, uint32_t n, uint32_t& v) {
  uint32_t val = 0, oct = 0, olen = 0, nd = 0, bad = (uint32_t)(n > 15u), lz = 0;
  for (uint32_t i = 0; i < 15; ++i) {
    const uint32_t c = x.b(i), in = (uint32_t)(i < n), dot = (uint32_t)(c == '.'), dig = (uint32_t)(c - '0' < 10u);
    const uint32_t ind = in & dot, ing = in & dig;
    bad |= (in & (dot | dig)) ^ in;
    bad |= ind & ((uint32_t)(olen == 0) | (uint32_t)(oct > 255u) | (uint32_t)(nd == 3));
    bad |= ing & ((uint32_t)(olen == 3) | ((uint32_t)(olen >= 1) & lz));
    lz = (ing & (uint32_t)(olen == 0)) ? (uint32_t)(c == '0') : lz;
    val = ind ? (val << 8) | oct : val;
    nd += ind;
    oct = ind ? 0u : (ing ? oct * 10u + (c - '0') : oct);
    olen = ind ? 0u : olen + ing;
  }
  bad |= (uint32_t)(olen == 0) | (uint32_t)(oct > 255u) | (uint32_t)(nd != 3);
  v = (val << 8) | oct;
  return !bad;
}
RSA_HD uint32_t b16_pack3(const B16& x) { return x.b(0) << 16 | x.b(1) << 8 | x.b(2); }
RSA_HD bool b16_ulll(const B16& x) { return is_upper(x.b(0)) && is_lower(x.b(1)) && is_lower(x.b(2)); }
constexpr uint32_t le4(char a, char b, char c, char d) {
  return (uint32_t)(uint8_t)a | (uint32_t)(uint8_t)b << 8 | (uint32_t)(uint8_t)c << 16 | (uint32_t)(uint8_t)d << 24;
}
// a name field [a, a + n): no '-' in it
template <class S>
RSA_HD bool name_no_dash(const S& s, uint32_t a, uint32_t n, const B16& first) {
  bool ok = !b16_has(first, n < 16 ? n : 16, '-');
  for (uint32_t o = 16; o < n && ok; o += 16) ok = !b16_has(bytes16(s, a + o), n - o < 16 ? n - o : 16, '-');
  return ok;
}
// a name field equal to an interface name (n <= RSA_IFC_NAME_MAX)
template <class S>
RSA_HD bool name_eq(const S& s, uint32_t a, uint32_t n, const B16& first, const char* name) {
  bool eq = true;
  for (uint32_t o = 0; o < n && eq; o += 16) {
    const B16 x = o ? bytes16(s, a + o) : first;
    B16 y{{0u, 0u, 0u, 0u}};
    for (uint32_t i = 0; i < 16; ++i) y.w[i >> 2] |= (o + i < n ? (uint32_t)(uint8_t)name[o + i] : 0u) << (8u * (i & 3u));
    eq = b16_eq(x, y, n - o < 16 ? n - o : 16);
  }
  return eq;
}

// parse_line for a line tpl::scan accepted, from its slots; false: leave the
// line to the general parse (everything parse_line would send to the host,
// and a '-' in an interface name, where the hit test must scan).  The fields
// are read as blocks (bytes16), all before the first test.
template <class S, class Q>
RSA_HD bool tpl_finish(const S& s, Q slot, const rsa_parse_ifc* ifcs, uint32_t n_ifcs, const rsa_parse_spell* spells,
                       uint32_t n_spells, rsa_tuple& tup, uint32_t& ts, uint32_t& d) {
  using namespace tpl;
  auto at = [&](uint32_t f) { return (uint32_t)slot[f] & 0xFFFFu; };
  auto len = [&](uint32_t f) { return ((uint32_t)slot[f] >> 16) & 0xFFu; };
  // two groups of blocks (fewer live registers at once): the header --
  // Mmm ... | Mmm D YYYY | TAG-d-dddddd | DIR PROTO -- then the addresses
  const B16 bM1 = bytes16(s, at(fM1)), bM2 = bytes16(s, at(fM2)), bTag = bytes16(s, at(fTAG)),
            bDir = bytes16(s, at(fDIR));
  const uint32_t m2 = b16_pack3(bM2);
  const uint32_t ltag = len(fTAG), tag = b16_pack3(bTag);
  bool ok = b16_ulll(bM1) && b16_ulll(bM2);
  ok = ok && (ltag == 3 ? (tag == pack3('A', 'S', 'A') || tag == pack3('P', 'I', 'X'))
                        : (tag == pack3('F', 'W', 'S') && bTag.b(3) == 'M'));
  const uint32_t ldir = len(fDIR);
  const bool inbound = ldir == 7 && bDir.w[0] == le4('i', 'n', 'b', 'o') && (bDir.w[1] & 0xFFFFFFu) == le4('u', 'n', 'd', 0);
  const bool outbound = ldir == 8 && bDir.w[0] == le4('o', 'u', 't', 'b') && bDir.w[1] == le4('o', 'u', 'n', 'd');
  ok = ok && (inbound || outbound);
  // PROTO follows DIR and one space
  const B16 bPr = outbound ? B16{{bDir.w[2] >> 8 | bDir.w[3] << 24, bDir.w[3] >> 8, 0u, 0u}}
                           : B16{{bDir.w[2], bDir.w[3], 0u, 0u}};
  const uint32_t proto = b16_pack3(bPr);
  const bool udp = proto == pack3('U', 'D', 'P');
  ok = ok && (udp || proto == pack3('T', 'C', 'P'));
  if (!ok) return false;
  // IF:IP/P (IP/P) to IF:IP/P
  const B16 bIf1 = bytes16(s, at(fIF1)), bIp1 = bytes16(s, at(fIP1)), bP1 = bytes16(s, at(fP1)),
            bIf2 = bytes16(s, at(fIF2)), bIp2 = bytes16(s, at(fIP2)), bP2 = bytes16(s, at(fP2));
  const uint32_t l1 = len(fIF1), l2 = len(fIF2);
  ok = ok && name_no_dash(s, at(fIF1), l1, bIf1) && name_no_dash(s, at(fIF2), l2, bIf2);   // '-' in a name
  uint32_t ip1 = 0, ip2 = 0;
  ok = ok && b16_ipv4(bIp1, len(fIP1), ip1) && b16_ipv4(bIp2, len(fIP2), ip2);   // not canonical quads
  const uint32_t lp1 = len(fP1), lp2 = len(fP2);
  const uint32_t p1 = b16_port(bP1, lp1), p2 = b16_port(bP2, lp2);
  ok = ok && p1 <= 65535u && p2 <= 65535u && (lp2 == 1 || bP2.b(0) != '0');   // long ports; TOPORT not canonical
  if (!ok) return false;
  const uint32_t src = inbound ? ip1 : ip2, dst = inbound ? ip2 : ip1;
  const uint32_t sp = inbound ? p1 : p2, dp = inbound ? p2 : p1;
  // the interface of the ingress side
  const uint32_t ia = inbound ? at(fIF1) : at(fIF2), il = inbound ? l1 : l2;
  const B16 bIf = inbound ? bIf1 : bIf2;
  int32_t found = -1;
  if (il > RSA_IFC_NAME_MAX) return false;
  for (uint32_t k = 0; k < n_ifcs && found < 0; ++k)
    if (ifcs[k].len == il && name_eq(s, ia, il, bIf, ifcs[k].name)) found = (int32_t)k;
  tup = rsa_tuple{0u, 0u, 0, 0, 0, 0, 0};
  ts = 0;
  if (found < 0) {
    d = RSA_LINE_NOACL;
    return true;
  }
  if (ifcs[found].kind == RSA_LINE_MISSING) {
    d = RSA_LINE_MISSING | ((uint32_t)found << 8);
    return true;
  }
  if (ifcs[found].kind != RSA_LINE_CLASSIFY) return false;
  const uint32_t lid = udp ? ifcs[found].list_udp : ifcs[found].list_tcp;
  if (lid == RSA_LIST_HOST) return false;
  // the reducer's fields: FROMIP = the first address, TOIP = the second, TOPORT = P2
  const B16 bSm = b16_shr(bTag, ltag - 3);   // "TAG-d-dddddd" from the tag's last 3 bytes: d at 4, dddddd at 6
  const uint32_t sev = bSm.b(4) - '0', msg = b16_num<6>(bSm, 6, 6);
  const bool hit = sev == 6 && (msg == 302013 || msg == 302015);
  uint32_t flags = RSA_F_VALID | RSA_F_BUILT | (hit ? RSA_F_HIT : 0u);
  // outbound: the reducer key is (IP1, IP2, P2) = (dst, src, sport) -- unless its
  // text equals the (src, dst, dport) one, which parse_line's first test takes
  if (outbound && !(ip1 == ip2 && lp1 == lp2 && b16_eq(bP1, bP2, lp1))) flags |= RSA_F_SWAP;
  if (hit) {
    // ts_code: HH:MM:SS of the syslog header, the device date's month, day, year
    const char* const months = "JanFebMarAprMayJunJulAugSepOctNovDec";
    int mo = -1;
    for (int k = 0; k < 12; ++k)
      if (m2 == pack3(months[3 * k], months[3 * k + 1], months[3 * k + 2])) mo = k;
    const uint32_t ld = len(fD2);   // "Mmm D YYYY" / "Mmm DD YYYY"
    const uint32_t day = b16_num<2>(bM2, 4, ld);
    const uint32_t y = ld == 1 ? b16_num<4>(bM2, 6, 4) : b16_num<4>(bM2, 7, 4);
    const B16 bHMS = bytes16(s, at(fHH));
    const uint32_t hh = b16_num<2>(bHMS, 0, 2), mm = b16_num<2>(bHMS, 3, 2), ss = b16_num<2>(bHMS, 6, 2);
    if (mo < 0 || y < RSA_TS_YEAR0 || y >= RSA_TS_YEAR0 + 128 || day > 31 || hh > 23 || mm > 59 || ss > 59)
      return false;
    ts = ((((y - RSA_TS_YEAR0) * 12u + (uint32_t)mo) * 32u + day) * 86400u) + hh * 3600u + mm * 60u + ss;
  }
  int32_t sid = -1;
  for (uint32_t k = 0; k < n_spells && sid < 0; ++k)
    if (spells[k].len == 3 && pack3(spells[k].word[0], spells[k].word[1], spells[k].word[2]) == proto)
      sid = (int32_t)k;
  if (sid < 0) return false;
  tup.src = src;
  tup.dst = dst;
  tup.sport = (uint16_t)sp;
  tup.dport = (uint16_t)dp;
  tup.list = (uint16_t)lid;
  tup.flags = (uint8_t)flags;
  tup.pspell = (uint8_t)sid;
  d = RSA_LINE_CLASSIFY;
  return true;
}

// ---- the reducer drop-in: one line of the sorted mapper stream
// (connlist-reducer.py:62-79,146-165)

RSA_HD bool is_py2ws(uint32_t c) { return c == ' ' || c - 9u < 5u; }   // Python 2 str.strip(): ' \t\n\v\f\r'

// The value of a mapper-stream line: byte i = byte o + i of the line.
template <class S>
struct SubLn {
  const S& s;
  uint32_t o;
  uint32_t n;
  RSA_HD uint32_t operator[](uint32_t i) const { return s[o + i]; }
};

// line.strip().split('\t', 1): the key is [a, t); false when the stripped
// line [a, b) has no tab (the reducer's ValueError "Unable to unpack" line)
template <class S>
RSA_HD bool key_span(const S& s, uint32_t& a, uint32_t& t, uint32_t& b) {
  a = 0;
  b = s.n;
  while (a < b && is_py2ws(s[a])) ++a;
  while (b > a && is_py2ws(s[b - 1])) --b;
  for (t = a; t < b; ++t)
    if (s[t] == '\t') return true;
  return false;
}

// The reducer's per-line fields: disposition (RSA_RED_* or RSA_LINE_HOST),
// tuple (src = FROMIP, dst = TOIP, dport = TOPORT, pspell, flags) and the
// timestamp code of a hit line whose value the BUILT regex matches.
template <bool kDefer = false, class S>
RSA_HD void reduce_line(const S& s, const rsa_parse_spell* spells, uint32_t n_spells, rsa_tuple& tup_out,
                        uint32_t& ts_out, uint32_t& d_out) {
  rsa_tuple tup = {0u, 0u, 0, 0, 0, 0, 0};
  uint32_t ts = 0, d = RSA_RED_NOISE;
  uint32_t a, t, b;
  if (key_span(s, a, t, b)) {
    d = RSA_RED_KEYED;
    const SubLn<S> v{s, t + 1, b - t - 1};
    uint32_t flags = 0;
    Reduced r;
    Mapped m;
    Hdr h;
    bool hit = false;
    const bool fast = gb_match(v, m, h) && built_template<!kDefer>(v, m, h, r, hit);   // the canonical form
    bool built = fast;
    if constexpr (kDefer) {
      if (!fast) {
        tup_out = rsa_tuple{0u, 0u, 0, 0, 0, 0, 0};
        ts_out = 0;
        d_out = kLineDefer;
        return;
      }
    } else {
      if (!fast) {
        hit = hit_test(v);
        built = built_search(v, r);
      }
    }
    if (hit) flags |= RSA_F_HIT;
    if (built) {
      flags |= RSA_F_BUILT;
      uint32_t vf = 0, vt = 0;
      const uint32_t pv = port_val(v, r.to_port);
      // the key is the text: canonical text <-> value is one to one
      if (!ipv4_canon(v, r.for_ip, vf) || !ipv4_canon(v, r.to_ip, vt) || !port_canon(v, r.to_port) || pv > 65535u)
        d = RSA_LINE_HOST;
      if (hit && !ts_code(v, r, ts)) d = RSA_LINE_HOST;
      int32_t sid = -1;
      const uint32_t wl = r.word.b - r.word.a;
      for (uint32_t k = 0; k < n_spells && sid < 0; ++k) {
        if (spells[k].len != wl) continue;
        bool eq = true;
        for (uint32_t c = 0; c < wl && eq; ++c) eq = v[r.word.a + c] == (uint8_t)spells[k].word[c];
        if (eq) sid = (int32_t)k;
      }
      if (sid < 0) d = RSA_LINE_HOST;
      tup.src = vf;
      tup.dst = vt;
      tup.dport = (uint16_t)pv;
      tup.pspell = (uint8_t)(sid < 0 ? 0 : sid);
    }
    tup.flags = (uint8_t)flags;
  }
  if (d != RSA_RED_KEYED) {
    tup = rsa_tuple{0u, 0u, 0, 0, 0, 0, 0};
    ts = 0;
  }
  tup_out = tup;
  ts_out = ts;
  d_out = d;
}

// Key bytes of two lines equal (both keyed): runs of equal keys.
template <class S1, class S2>
RSA_HD bool same_key(const S1& x, const S2& y) {
  uint32_t xa, xt, xb, ya, yt, yb;
  if (!key_span(x, xa, xt, xb) || !key_span(y, ya, yt, yb) || xt - xa != yt - ya) return false;
  for (uint32_t i = 0; i < xt - xa; ++i)
    if (x[xa + i] != y[ya + i]) return false;
  return true;
}

#undef RSA_HD

}  // namespace rsa_text

#endif
