// SPDX-License-Identifier: Apache-2.0
// base64 (RFC 4648) for the etcd-v3 JSON gateway wire format (keys/values
// are base64-encoded bytes there).
#include "base64.h"

namespace pdo {

static const char kAlpha[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string b64encode(const std::string& in) {
  std::string out;
  out.reserve((in.size() + 2) / 3 * 4);
  size_t i = 0;
  while (i + 2 < in.size()) {
    unsigned v = ((unsigned char)in[i] << 16) | ((unsigned char)in[i + 1] << 8) | (unsigned char)in[i + 2];
    out.push_back(kAlpha[(v >> 18) & 63]);
    out.push_back(kAlpha[(v >> 12) & 63]);
    out.push_back(kAlpha[(v >> 6) & 63]);
    out.push_back(kAlpha[v & 63]);
    i += 3;
  }
  if (i + 1 == in.size()) {
    unsigned v = (unsigned char)in[i] << 16;
    out.push_back(kAlpha[(v >> 18) & 63]);
    out.push_back(kAlpha[(v >> 12) & 63]);
    out += "==";
  } else if (i + 2 == in.size()) {
    unsigned v = ((unsigned char)in[i] << 16) | ((unsigned char)in[i + 1] << 8);
    out.push_back(kAlpha[(v >> 18) & 63]);
    out.push_back(kAlpha[(v >> 12) & 63]);
    out.push_back(kAlpha[(v >> 6) & 63]);
    out.push_back('=');
  }
  return out;
}

bool b64decode(const std::string& in, std::string* out) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+' || c == '-') return 62;
    if (c == '/' || c == '_') return 63;
    return -1;
  };
  out->clear();
  unsigned buf = 0;
  int bits = 0;
  for (char c : in) {
    if (c == '=' || c == '\n' || c == '\r') continue;
    int v = val(c);
    if (v < 0) return false;
    buf = (buf << 6) | (unsigned)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      out->push_back((char)((buf >> bits) & 0xff));
    }
  }
  return true;
}

}  // namespace pdo
