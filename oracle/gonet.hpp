// oracle/gonet.hpp — restatement of the Go 1.16 standard-library `net` functions that the
// reference calls on the verdict path (test infrastructure only).
//
// Third-party algorithm: Go stdlib `net`, pinned to Go 1.16 (reference go.mod:3,
// .github/workflows/go.yml:17).  Call sites in the reference:
//   pkg/kube/ipaddress.go:10-20  IsIPInCIDR   -> net.ParseCIDR, net.ParseIP, (*IPNet).Contains
//   pkg/kube/ipaddress.go:42-46  MakeIPV4CIDR -> net.CIDRMask, net.ParseIP, IP.Mask
// Restated from the published Go 1.16 net/ip.go algorithm: parseIPv4 (leading zeros
// ACCEPTED in 1.16), parseIPv6 (embedded dotted quad, "::" ellipsis), ParseCIDR (mask via
// dtoi, IPv4 tried first), IP.Mask, IP.To4 and IPNet.Contains / networkNumberAndMask.
// IPs are byte vectors whose length (4 or 16) matters exactly as in Go.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace gonet {

using IP = std::vector<uint8_t>;  // empty == Go nil

static const int kBig = 0xFFFFFF;

// net/parse.go dtoi: decimal to integer, returns (n, chars consumed, ok)
inline void dtoi(const std::string& s, size_t off, int& n, size_t& i, bool& ok) {
  n = 0;
  for (i = 0; off + i < s.size() && s[off + i] >= '0' && s[off + i] <= '9'; i++) {
    n = n * 10 + (s[off + i] - '0');
    if (n >= kBig) {
      n = kBig;
      ok = false;
      return;
    }
  }
  ok = i != 0;
}

// net/parse.go xtoi: hexadecimal to integer
inline void xtoi(const std::string& s, size_t off, int& n, size_t& i, bool& ok) {
  n = 0;
  for (i = 0; off + i < s.size(); i++) {
    char c = s[off + i];
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
    else break;
    n = n * 16 + d;
    if (n >= kBig) {
      ok = false;
      n = 0;
      return;
    }
  }
  ok = i != 0;
}

inline IP ipv4(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {
  IP p(16, 0);
  p[10] = 0xff;
  p[11] = 0xff;
  p[12] = a;
  p[13] = b;
  p[14] = c;
  p[15] = d;
  return p;
}

// net/ip.go parseIPv4 (Go 1.16: no leading-zero rejection)
inline IP parse_ipv4(const std::string& s0) {
  uint8_t p[4];
  size_t pos = 0;
  const std::string& s = s0;
  for (int i = 0; i < 4; i++) {
    if (pos >= s.size()) return {};
    if (i > 0) {
      if (s[pos] != '.') return {};
      pos++;
    }
    int n;
    size_t c;
    bool ok;
    dtoi(s, pos, n, c, ok);
    if (!ok || n > 0xFF) return {};
    pos += c;
    p[i] = uint8_t(n);
  }
  if (pos != s.size()) return {};
  return ipv4(p[0], p[1], p[2], p[3]);
}

// net/ip.go parseIPv6 (no zone)
inline IP parse_ipv6(const std::string& s0) {
  IP ip(16, 0);
  int ellipsis = -1;
  std::string s = s0;
  if (s.size() >= 2 && s[0] == ':' && s[1] == ':') {
    ellipsis = 0;
    s = s.substr(2);
    if (s.empty()) return ip;
  }
  int i = 0;
  while (i < 16) {
    int n;
    size_t c;
    bool ok;
    xtoi(s, 0, n, c, ok);
    if (!ok || n > 0xFFFF) return {};
    if (c < s.size() && s[c] == '.') {
      if (ellipsis < 0 && i != 16 - 4) return {};
      if (i + 4 > 16) return {};
      IP ip4 = parse_ipv4(s);
      if (ip4.empty()) return {};
      ip[i] = ip4[12];
      ip[i + 1] = ip4[13];
      ip[i + 2] = ip4[14];
      ip[i + 3] = ip4[15];
      s.clear();
      i += 4;
      break;
    }
    ip[i] = uint8_t(n >> 8);
    ip[i + 1] = uint8_t(n);
    i += 2;
    s = s.substr(c);
    if (s.empty()) break;
    if (s[0] != ':' || s.size() == 1) return {};
    s = s.substr(1);
    if (s[0] == ':') {
      if (ellipsis >= 0) return {};
      ellipsis = i;
      s = s.substr(1);
      if (s.empty()) break;
    }
  }
  if (!s.empty()) return {};
  if (i < 16) {
    if (ellipsis < 0) return {};
    int n = 16 - i;
    for (int j = i - 1; j >= ellipsis; j--) ip[j + n] = ip[j];
    for (int j = ellipsis + n - 1; j >= ellipsis; j--) ip[j] = 0;
  } else if (ellipsis >= 0) {
    return {};
  }
  return ip;
}

// net/ip.go ParseIP
inline IP ParseIP(const std::string& s) {
  for (char c : s) {
    if (c == '.') return parse_ipv4(s);
    if (c == ':') return parse_ipv6(s);
  }
  return {};
}

// net/ip.go CIDRMask
inline IP CIDRMask(int ones, int bits) {
  if (bits != 32 && bits != 128) return {};
  if (ones < 0 || ones > bits) return {};
  int l = bits / 8;
  IP m(l, 0);
  int n = ones;
  for (int i = 0; i < l; i++) {
    if (n >= 8) {
      m[i] = 0xff;
      n -= 8;
      continue;
    }
    m[i] = uint8_t(~(0xff >> n));
    n = 0;
  }
  return m;
}

inline bool is_v4_in_v6(const IP& ip) {
  if (ip.size() != 16) return false;
  for (int i = 0; i < 10; i++)
    if (ip[i] != 0) return false;
  return ip[10] == 0xff && ip[11] == 0xff;
}

// net/ip.go To4
inline IP To4(const IP& ip) {
  if (ip.size() == 4) return ip;
  if (is_v4_in_v6(ip)) return IP(ip.begin() + 12, ip.end());
  return {};
}

// net/ip.go IP.Mask
inline IP Mask(IP ip, IP mask) {
  if (mask.size() == 16 && ip.size() == 4) {
    bool allff = true;
    for (int i = 0; i < 12; i++) allff = allff && mask[i] == 0xff;
    if (allff) mask = IP(mask.begin() + 12, mask.end());
  }
  if (mask.size() == 4 && ip.size() == 16 && is_v4_in_v6(ip)) ip = IP(ip.begin() + 12, ip.end());
  if (ip.size() != mask.size()) return {};
  IP out(ip.size());
  for (size_t i = 0; i < ip.size(); i++) out[i] = ip[i] & mask[i];
  return out;
}

struct IPNet {
  IP ip;
  IP mask;
};

// net/ip.go ParseCIDR; returns false on error (Go returns *ParseError)
inline bool ParseCIDR(const std::string& s, IPNet& out) {
  size_t slash = s.find('/');
  if (slash == std::string::npos) return false;
  std::string addr = s.substr(0, slash), mask = s.substr(slash + 1);
  int iplen = 4;
  IP ip = parse_ipv4(addr);
  if (ip.empty()) {
    iplen = 16;
    ip = parse_ipv6(addr);
  }
  int n;
  size_t i;
  bool ok;
  dtoi(mask, 0, n, i, ok);
  if (ip.empty() || !ok || i != mask.size() || n < 0 || n > 8 * iplen) return false;
  IP m = CIDRMask(n, 8 * iplen);
  out.ip = Mask(ip, m);
  out.mask = m;
  return true;
}

// net/ip.go networkNumberAndMask + IPNet.Contains
inline bool Contains(const IPNet& n, IP ip) {
  IP nn = To4(n.ip);
  if (nn.empty()) {
    nn = n.ip;
    if (nn.size() != 16) return false;
  }
  IP m = n.mask;
  if (m.size() == 4) {
    if (nn.size() != 4) return false;
  } else if (m.size() == 16) {
    if (nn.size() == 4) m = IP(m.begin() + 12, m.end());
  } else {
    return false;
  }
  IP x = To4(ip);
  if (!x.empty()) ip = x;
  if (ip.size() != nn.size()) return false;
  for (size_t i = 0; i < ip.size(); i++)
    if ((nn[i] & m[i]) != (ip[i] & m[i])) return false;
  return true;
}

// net/ip.go IP.String (used only by MakeIPV4CIDR for IPv4 results in tests)
inline std::string IPv4String(const IP& ip4) {
  return std::to_string(ip4[0]) + "." + std::to_string(ip4[1]) + "." + std::to_string(ip4[2]) + "." +
         std::to_string(ip4[3]);
}

}  // namespace gonet
