// SPDX-License-Identifier: Apache-2.0
#include "quantity.h"

#include <cctype>
#include <cstdlib>
#include <string>

namespace pdo {

static std::string i128_to_string(__int128 v) {
  if (v == 0) return "0";
  bool neg = v < 0;
  if (neg) v = -v;
  std::string s;
  while (v > 0) {
    s.push_back((char)('0' + (int)(v % 10)));
    v /= 10;
  }
  if (neg) s.push_back('-');
  return std::string(s.rbegin(), s.rend());
}

bool Quantity::parse(const std::string& in, Quantity* out) {
  std::string s;
  for (char c : in)
    if (!isspace((unsigned char)c)) s.push_back(c);
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[i] == '+' || s[i] == '-') neg = s[i++] == '-';
  std::string ip, fp;
  while (i < s.size() && isdigit((unsigned char)s[i])) ip.push_back(s[i++]);
  if (i < s.size() && s[i] == '.') {
    ++i;
    while (i < s.size() && isdigit((unsigned char)s[i])) fp.push_back(s[i++]);
  }
  if (ip.empty() && fp.empty()) return false;
  std::string suf = s.substr(i);
  // mantissa as an exact integer × 10^-len(fp)
  __int128 mant = 0;
  for (char c : ip + fp) mant = mant * 10 + (c - '0');
  int dec_exp = -(int)fp.size();
  __int128 mul_bin = 1;
  Format fmt = Format::DecimalSI;
  if (suf.empty()) {
  } else if (suf == "m") dec_exp -= 3;
  else if (suf == "k") dec_exp += 3;
  else if (suf == "M") dec_exp += 6;
  else if (suf == "G") dec_exp += 9;
  else if (suf == "T") dec_exp += 12;
  else if (suf == "P") dec_exp += 15;
  else if (suf == "E") dec_exp += 18;
  else if (suf == "Ki" || suf == "Mi" || suf == "Gi" || suf == "Ti" || suf == "Pi" || suf == "Ei") {
    const char* order = "KMGTPE";
    int k = 0;
    while (order[k] != suf[0]) ++k;
    for (int t = 0; t <= k; ++t) mul_bin *= 1024;
    fmt = Format::BinarySI;
  } else if (suf[0] == 'e' || suf[0] == 'E') {
    char* endp = nullptr;
    long e = strtol(suf.c_str() + 1, &endp, 10);
    if (!endp || *endp) return false;
    dec_exp += (int)e;
    fmt = Format::DecimalExponent;
  } else {
    return false;
  }
  // milli = mant * mul_bin * 10^(dec_exp + 3), rounded up (Go rounds up to the scale)
  __int128 v = mant * mul_bin;
  int e3 = dec_exp + 3;
  if (e3 >= 0) {
    for (int t = 0; t < e3; ++t) v *= 10;
  } else {
    __int128 d = 1;
    for (int t = 0; t < -e3; ++t) d *= 10;
    v = (v + d - 1) / d;
  }
  out->milli_ = neg ? -v : v;
  out->fmt_ = fmt;
  return true;
}

std::string Quantity::str() const {
  __int128 m = milli_;
  if (m == 0) return "0";
  const bool integral = (m % 1000) == 0;
  if (!integral) {
    // milli form is exact
    return i128_to_string(m) + "m";
  }
  __int128 v = m / 1000;
  if (fmt_ == Format::BinarySI) {
    static const char* suf[] = {"", "Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
    int k = 0;
    while (k < 6 && v != 0 && v % 1024 == 0) {
      v /= 1024;
      ++k;
    }
    return i128_to_string(v) + suf[k];
  }
  if (fmt_ == Format::DecimalExponent) {
    int e = 0;
    while (v != 0 && v % 1000 == 0) {
      v /= 1000;
      e += 3;
    }
    return e ? i128_to_string(v) + "e" + std::to_string(e) : i128_to_string(v);
  }
  static const char* suf[] = {"", "k", "M", "G", "T", "P", "E"};
  int k = 0;
  while (k < 6 && v != 0 && v % 1000 == 0) {
    v /= 1000;
    ++k;
  }
  return i128_to_string(v) + suf[k];
}

}  // namespace pdo
