// _m2k_sshkey: private SSH keys parsed, decrypted and re-encoded in process.
//
// The reference reads a user's private key with golang.org/x/crypto/ssh
// (x/crypto@c8d3bf9c5392, go.mod:37) and writes it back as PEM for Tekton's
// git-init (internal/common/sshkeys/sshkeys.go:170-232):
//
//   key, err := ssh.ParseRawPrivateKey(fileBytes)            // PassphraseMissingError -> ask
//   key, err = ssh.ParseRawPrivateKeyWithPassphrase(fileBytes, password)
//   *rsa.PrivateKey   -> x509.MarshalPKCS1PrivateKey -> "RSA PRIVATE KEY"
//   *ecdsa.PrivateKey -> x509.MarshalECPrivateKey    -> "EC PRIVATE KEY"
//   anything else     -> "Unknown key type [%T]"
//
// This file does the same without an external program:
//   * encoding/pem Decode (first block, headers, base64 body);
//   * "OPENSSH PRIVATE KEY" (openssh-key-v1): cipher "none", or aes256-ctr /
//     aes256-cbc keyed by bcrypt_pbkdf (Blowfish's expensive key schedule,
//     SHA-512; x/crypto/ssh/internal/bcrypt_pbkdf), check-int test,
//     ssh-rsa / ecdsa-sha2-nistp{256,384,521} / ssh-ed25519 sections;
//   * legacy PEM with Proc-Type/DEK-Info (x509.DecryptPEMBlock: MD5
//     EVP_BytesToKey, DES-CBC, DES-EDE3-CBC, AES-{128,192,256}-CBC, RFC 1423
//     padding as the password check);
//   * PKCS#1, PKCS#8 and SEC1 DER (x509.Parse*PrivateKey), DSA;
//   * output: PKCS#1 RSA with the CRT values recomputed (rsa.Precompute) or
//     SEC1 EC with the public point recomputed from d (curve.ScalarBaseMult).
//
// OpenSSL's libcrypto provides the block ciphers, digests, bignums and curve
// arithmetic; Blowfish (for bcrypt) is here, its tables generated from pi
// (gen_blowfish_pi.py).  Built as its own extension so that only a command
// that loads a key maps libcrypto (utils/sshkeys.py imports it on use).

#include <pybind11/pybind11.h>

#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "blowfish_pi.h"

namespace py = pybind11;

namespace {

using Bytes = std::string;

struct GoError {
  std::string msg;
};
struct PassphraseMissing {};

[[noreturn]] void fail(const std::string& m) { throw GoError{m}; }

// strconv.Quote of an ASCII-ish string (the texts Go prints with %q here).
std::string go_quote(const std::string& s) {
  static const char* hex = "0123456789abcdef";
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += static_cast<char>(c);
    } else if (c >= 0x20 && c < 0x7f) {
      o += static_cast<char>(c);
    } else if (c == '\n') {
      o += "\\n";
    } else if (c == '\t') {
      o += "\\t";
    } else if (c == '\r') {
      o += "\\r";
    } else {
      o += "\\x";
      o += hex[c >> 4];
      o += hex[c & 15];
    }
  }
  return o + "\"";
}

// ---------------------------------------------------------------------------
// RAII for OpenSSL objects
// ---------------------------------------------------------------------------

struct BnFree {
  void operator()(BIGNUM* b) const { BN_clear_free(b); }
};
using Bn = std::unique_ptr<BIGNUM, BnFree>;
struct CtxFree {
  void operator()(BN_CTX* c) const { BN_CTX_free(c); }
};
struct GroupFree {
  void operator()(EC_GROUP* g) const { EC_GROUP_free(g); }
};
struct PointFree {
  void operator()(EC_POINT* p) const { EC_POINT_free(p); }
};
struct CipherCtxFree {
  void operator()(EVP_CIPHER_CTX* c) const { EVP_CIPHER_CTX_free(c); }
};

Bn bn_bin(const Bytes& b) {
  Bn r(BN_bin2bn(reinterpret_cast<const unsigned char*>(b.data()), static_cast<int>(b.size()), nullptr));
  if (!r) fail("out of memory");
  return r;
}

Bn bn_new() {
  Bn r(BN_new());
  if (!r) fail("out of memory");
  return r;
}

Bytes bn_bytes(const BIGNUM* b) {
  Bytes out(static_cast<size_t>(BN_num_bytes(b)), '\0');
  BN_bn2bin(b, reinterpret_cast<unsigned char*>(&out[0]));
  return out;
}

// ---------------------------------------------------------------------------
// base64 (encoding/base64 StdEncoding; '\r' and '\n' are skipped on decode)
// ---------------------------------------------------------------------------

const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

bool b64_decode(const std::string& in, Bytes& out) {
  int vals[256];
  for (int& v : vals) v = -1;
  for (int i = 0; i < 64; i++) vals[static_cast<unsigned char>(kB64[i])] = i;
  std::vector<int> q;
  q.reserve(in.size());
  size_t pad = 0;
  for (unsigned char c : in) {
    if (c == '\r' || c == '\n') continue;
    if (c == '=') {
      pad++;
      q.push_back(0);
      continue;
    }
    if (pad || vals[c] < 0) return false;  // data after padding, or a bad character
    q.push_back(vals[c]);
  }
  if (q.size() % 4 != 0 || pad > 2) return false;
  out.clear();
  for (size_t i = 0; i < q.size(); i += 4) {
    uint32_t v = (q[i] << 18) | (q[i + 1] << 12) | (q[i + 2] << 6) | q[i + 3];
    out += static_cast<char>(v >> 16);
    out += static_cast<char>((v >> 8) & 0xff);
    out += static_cast<char>(v & 0xff);
  }
  out.resize(out.size() - pad);
  return true;
}

std::string b64_encode(const Bytes& in) {
  std::string o;
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    uint32_t v = (static_cast<unsigned char>(in[i]) << 16) | (static_cast<unsigned char>(in[i + 1]) << 8) |
                 static_cast<unsigned char>(in[i + 2]);
    o += kB64[v >> 18];
    o += kB64[(v >> 12) & 63];
    o += kB64[(v >> 6) & 63];
    o += kB64[v & 63];
  }
  if (i + 1 == in.size()) {
    uint32_t v = static_cast<unsigned char>(in[i]) << 16;
    o += kB64[v >> 18];
    o += kB64[(v >> 12) & 63];
    o += "==";
  } else if (i + 2 == in.size()) {
    uint32_t v = (static_cast<unsigned char>(in[i]) << 16) | (static_cast<unsigned char>(in[i + 1]) << 8);
    o += kB64[v >> 18];
    o += kB64[(v >> 12) & 63];
    o += kB64[(v >> 6) & 63];
    o += '=';
  }
  return o;
}

// pem.EncodeToMemory with no headers: 64-column base64 lines.
std::string pem_encode(const std::string& type, const Bytes& der) {
  std::string b = b64_encode(der);
  std::string o = "-----BEGIN " + type + "-----\n";
  for (size_t i = 0; i < b.size(); i += 64) o += b.substr(i, 64) + "\n";
  return o + "-----END " + type + "-----\n";
}

// ---------------------------------------------------------------------------
// encoding/pem Decode
// ---------------------------------------------------------------------------

struct PemBlock {
  std::string type;
  std::vector<std::pair<std::string, std::string>> headers;  // in order; lookups take the last
  Bytes bytes;

  const std::string* header(const std::string& k) const {
    const std::string* v = nullptr;
    for (auto& h : headers)
      if (h.first == k) v = &h.second;
    return v;
  }
};

std::string trim_right(const std::string& s, const char* set) {
  size_t e = s.find_last_not_of(set);
  return e == std::string::npos ? std::string() : s.substr(0, e + 1);
}

std::string trim_space(const std::string& s) {
  const char* ws = " \t\r\n\v\f";
  size_t b = s.find_first_not_of(ws);
  if (b == std::string::npos) return std::string();
  size_t e = s.find_last_not_of(ws);
  return s.substr(b, e - b + 1);
}

// pem.go getLine: up to '\n' (a '\r' before it dropped), trailing spaces and tabs trimmed.
std::pair<std::string, std::string> get_line(const std::string& data) {
  size_t i = data.find('\n');
  size_t j;
  if (i == std::string::npos) {
    i = j = data.size();
  } else {
    j = i + 1;
    if (i > 0 && data[i - 1] == '\r') i--;
  }
  return {trim_right(data.substr(0, i), " \t"), data.substr(j)};
}

bool pem_decode_one(const std::string& data, PemBlock& p, std::string& rest_out, std::string& err_rest) {
  static const std::string kStart = "\n-----BEGIN ", kEnd = "\n-----END ", kEol = "-----";
  std::string rest;
  if (data.compare(0, kStart.size() - 1, kStart, 1, std::string::npos) == 0) {
    rest = data.substr(kStart.size() - 1);
  } else {
    size_t i = data.find(kStart);
    if (i == std::string::npos) {
      err_rest.clear();
      return false;
    }
    rest = data.substr(i + kStart.size());
  }
  auto tl = get_line(rest);
  std::string type_line = tl.first;
  rest = tl.second;
  if (type_line.size() < kEol.size() || type_line.compare(type_line.size() - kEol.size(), kEol.size(), kEol) != 0) {
    err_rest = rest;
    return false;
  }
  type_line.resize(type_line.size() - kEol.size());
  p.type = type_line;
  p.headers.clear();
  while (true) {
    if (rest.empty()) {
      err_rest.clear();
      return false;
    }
    auto ln = get_line(rest);
    size_t c = ln.first.find(':');
    if (c == std::string::npos) break;
    p.headers.emplace_back(trim_space(ln.first.substr(0, c)), trim_space(ln.first.substr(c + 1)));
    rest = ln.second;
  }
  size_t end_index, end_trailer;
  if (p.headers.empty() && rest.compare(0, kEnd.size() - 1, kEnd, 1, std::string::npos) == 0) {
    end_index = 0;
    end_trailer = kEnd.size() - 1;
  } else {
    end_index = rest.find(kEnd);
    if (end_index == std::string::npos) {
      err_rest = rest;
      return false;
    }
    end_trailer = end_index + kEnd.size();
  }
  std::string trailer = rest.substr(end_trailer);
  size_t trailer_len = type_line.size() + kEol.size();
  if (trailer.size() < trailer_len) {
    err_rest = rest;
    return false;
  }
  std::string rest_of_end = trailer.substr(trailer_len);
  trailer.resize(trailer_len);
  if (trailer.compare(0, type_line.size(), type_line) != 0 ||
      trailer.compare(trailer.size() - kEol.size(), kEol.size(), kEol) != 0) {
    err_rest = rest;
    return false;
  }
  if (!get_line(rest_of_end).first.empty()) {
    err_rest = rest;
    return false;
  }
  std::string b64;
  for (char ch : rest.substr(0, end_index))
    if (ch != ' ' && ch != '\t') b64 += ch;
  if (!b64_decode(b64, p.bytes)) {
    err_rest = rest;
    return false;
  }
  rest_out = get_line(rest.substr(end_index + kEnd.size() - 1)).second;
  return true;
}

// pem.Decode: the first well-formed block (a malformed one is skipped, as
// decodeError retries on the rest).
bool pem_decode(const std::string& data, PemBlock& p) {
  std::string cur = data, rest, err_rest;
  for (int guard = 0; guard < 100000; guard++) {
    if (pem_decode_one(cur, p, rest, err_rest)) return true;
    if (err_rest.empty() || err_rest.size() >= cur.size()) return false;
    cur = err_rest;
  }
  return false;
}

// ---------------------------------------------------------------------------
// DER (encoding/asn1 subset: what the private-key structures use)
// ---------------------------------------------------------------------------

struct Der {
  const Bytes& b;
  size_t i, end;
  explicit Der(const Bytes& buf) : b(buf), i(0), end(buf.size()) {}
  Der(const Bytes& buf, size_t s, size_t e) : b(buf), i(s), end(e) {}

  bool done() const { return i >= end; }
  int peek_tag() const { return i < end ? static_cast<unsigned char>(b[i]) : -1; }

  // One TLV: its tag and the [start, stop) of its contents.
  void read(int& tag, size_t& s, size_t& e) {
    if (i + 2 > end) fail("asn1: syntax error: data truncated");
    tag = static_cast<unsigned char>(b[i++]);
    if ((tag & 0x1f) == 0x1f) fail("asn1: syntax error: long-form tags are not supported here");
    size_t len = static_cast<unsigned char>(b[i++]);
    if (len & 0x80) {
      size_t n = len & 0x7f;
      if (n == 0 || n > 4) fail("asn1: syntax error: indefinite or too long length");
      if (i + n > end) fail("asn1: syntax error: data truncated");
      if (b[i] == 0) fail("asn1: structure error: superfluous leading zeros in length");
      len = 0;
      for (size_t k = 0; k < n; k++) len = (len << 8) | static_cast<unsigned char>(b[i++]);
      if (len < 0x80) fail("asn1: structure error: non-minimal length");
    }
    if (i + len > end) fail("asn1: syntax error: data truncated");
    s = i;
    e = i + len;
    i = e;
  }

  Der enter(int want) {
    int tag;
    size_t s, e;
    read(tag, s, e);
    if (tag != want) fail("asn1: structure error: tags don't match");
    return Der(b, s, e);
  }

  Bytes raw(int want) {
    int tag;
    size_t s, e;
    read(tag, s, e);
    if (tag != want) fail("asn1: structure error: tags don't match");
    return b.substr(s, e - s);
  }

  // INTEGER -> positive bignum (a negative value is rejected by the callers' checks)
  Bn integer(bool* negative = nullptr) {
    Bytes v = raw(0x02);
    if (v.empty()) fail("asn1: syntax error: empty integer");
    if (v.size() > 1 && ((v[0] == 0 && !(v[1] & 0x80)) || (static_cast<unsigned char>(v[0]) == 0xff && (v[1] & 0x80))))
      fail("asn1: structure error: integer not minimally-encoded");
    bool neg = (v[0] & 0x80) != 0;
    if (negative) *negative = neg;
    if (neg) return bn_new();  // value unused: the caller reports the sign
    return bn_bin(v);
  }

  int64_t small_int() {
    Bytes v = raw(0x02);
    if (v.empty()) fail("asn1: syntax error: empty integer");
    if (v.size() > 8) fail("asn1: structure error: integer too large");
    uint64_t r = (v[0] & 0x80) ? ~uint64_t{0} : 0;  // sign-extended, shifted unsigned (no UB)
    for (unsigned char c : v) r = (r << 8) | c;
    return static_cast<int64_t>(r);
  }

  std::string oid() {
    Bytes v = raw(0x06);
    if (v.empty()) fail("asn1: syntax error: zero length OBJECT IDENTIFIER");
    std::string o;
    uint64_t acc = 0;
    bool first = true;
    for (unsigned char c : v) {
      acc = (acc << 7) | (c & 0x7f);
      if (!(c & 0x80)) {
        if (first) {
          uint64_t a = acc < 80 ? acc / 40 : 2;
          o = std::to_string(a) + "." + std::to_string(acc - 40 * a);
          first = false;
        } else {
          o += "." + std::to_string(acc);
        }
        acc = 0;
      }
    }
    return o;
  }
};

Bytes der_len(size_t n) {
  Bytes o;
  if (n < 0x80) {
    o += static_cast<char>(n);
  } else {
    Bytes l;
    while (n) {
      l.insert(l.begin(), static_cast<char>(n & 0xff));
      n >>= 8;
    }
    o += static_cast<char>(0x80 | l.size());
    o += l;
  }
  return o;
}

Bytes der_tlv(int tag, const Bytes& content) { return Bytes(1, static_cast<char>(tag)) + der_len(content.size()) + content; }

Bytes der_int(const BIGNUM* v) {
  Bytes b = bn_bytes(v);
  if (b.empty() || (b[0] & 0x80)) b.insert(b.begin(), '\0');
  return der_tlv(0x02, b);
}

Bytes der_small_int(int v) { return der_tlv(0x02, Bytes(1, static_cast<char>(v))); }

Bytes der_oid(const std::string& dotted) {
  std::vector<uint64_t> arcs;
  size_t p = 0;
  while (p <= dotted.size()) {
    size_t q = dotted.find('.', p);
    if (q == std::string::npos) q = dotted.size();
    arcs.push_back(std::stoull(dotted.substr(p, q - p)));
    p = q + 1;
  }
  Bytes o;
  auto put = [&o](uint64_t v) {
    Bytes t(1, static_cast<char>(v & 0x7f));
    v >>= 7;
    while (v) {
      t.insert(t.begin(), static_cast<char>(0x80 | (v & 0x7f)));
      v >>= 7;
    }
    o += t;
  };
  put(arcs[0] * 40 + arcs[1]);
  for (size_t k = 2; k < arcs.size(); k++) put(arcs[k]);
  return der_tlv(0x06, o);
}

// ---------------------------------------------------------------------------
// Keys
// ---------------------------------------------------------------------------

struct Curve {
  const char* oid;
  int nid;
  const char* ssh_name;
};
const Curve kCurves[] = {
    {"1.3.132.0.33", NID_secp224r1, ""},
    {"1.2.840.10045.3.1.7", NID_X9_62_prime256v1, "nistp256"},
    {"1.3.132.0.34", NID_secp384r1, "nistp384"},
    {"1.3.132.0.35", NID_secp521r1, "nistp521"},
};

struct Key {
  enum Kind { RSA, EC, OTHER } kind = OTHER;
  Bn n, e, d, p, q;       // RSA
  const Curve* curve = nullptr;  // EC
  Bn ec_d;
  std::string go_type;    // OTHER: the %T text
};

const BIGNUM* one() { return BN_value_one(); }

// rsa.PrivateKey.Validate (two primes) with checkPub.
void rsa_validate(const Key& k) {
  std::unique_ptr<BN_CTX, CtxFree> ctx(BN_CTX_new());
  if (BN_num_bits(k.e.get()) > 31) fail("crypto/rsa: public exponent too large");
  if (BN_cmp(k.e.get(), BN_value_one()) <= 0) fail("crypto/rsa: public exponent too small");
  if (BN_cmp(k.p.get(), one()) <= 0 || BN_cmp(k.q.get(), one()) <= 0) fail("crypto/rsa: invalid prime value");
  Bn mod = bn_new();
  BN_mul(mod.get(), k.p.get(), k.q.get(), ctx.get());
  if (BN_cmp(mod.get(), k.n.get()) != 0) fail("crypto/rsa: invalid modulus");
  Bn de = bn_new(), pm1 = bn_new(), r = bn_new();
  BN_mul(de.get(), k.e.get(), k.d.get(), ctx.get());
  for (const BIGNUM* prime : {k.p.get(), k.q.get()}) {
    BN_sub(pm1.get(), prime, one());
    BN_mod(r.get(), de.get(), pm1.get(), ctx.get());
    if (!BN_is_one(r.get())) fail("crypto/rsa: invalid exponents");
  }
}

// x509.MarshalPKCS1PrivateKey (Precompute: Dp, Dq, Qinv from D, P, Q).
std::string rsa_pem(const Key& k) {
  std::unique_ptr<BN_CTX, CtxFree> ctx(BN_CTX_new());
  Bn pm1 = bn_new(), qm1 = bn_new(), dp = bn_new(), dq = bn_new(), qinv = bn_new();
  BN_sub(pm1.get(), k.p.get(), one());
  BN_sub(qm1.get(), k.q.get(), one());
  BN_mod(dp.get(), k.d.get(), pm1.get(), ctx.get());
  BN_mod(dq.get(), k.d.get(), qm1.get(), ctx.get());
  if (!BN_mod_inverse(qinv.get(), k.q.get(), k.p.get(), ctx.get())) fail("crypto/rsa: invalid prime value");
  Bytes body = der_small_int(0) + der_int(k.n.get()) + der_int(k.e.get()) + der_int(k.d.get()) + der_int(k.p.get()) +
               der_int(k.q.get()) + der_int(dp.get()) + der_int(dq.get()) + der_int(qinv.get());
  return pem_encode("RSA PRIVATE KEY", der_tlv(0x30, body));
}

// (order bytes, uncompressed public point d*G) of an EC key.
void ec_public(const Key& k, size_t& order_len, Bytes& point) {
  std::unique_ptr<EC_GROUP, GroupFree> g(EC_GROUP_new_by_curve_name(k.curve->nid));
  std::unique_ptr<BN_CTX, CtxFree> ctx(BN_CTX_new());
  if (!g) fail("x509: unknown elliptic curve");
  Bn order = bn_new();
  EC_GROUP_get_order(g.get(), order.get(), ctx.get());
  order_len = static_cast<size_t>((BN_num_bits(order.get()) + 7) / 8);
  std::unique_ptr<EC_POINT, PointFree> pub(EC_POINT_new(g.get()));
  if (!EC_POINT_mul(g.get(), pub.get(), k.ec_d.get(), nullptr, nullptr, ctx.get())) fail("ecdsa: scalar mult failed");
  size_t n = EC_POINT_point2oct(g.get(), pub.get(), POINT_CONVERSION_UNCOMPRESSED, nullptr, 0, ctx.get());
  point.assign(n, '\0');
  EC_POINT_point2oct(g.get(), pub.get(), POINT_CONVERSION_UNCOMPRESSED, reinterpret_cast<unsigned char*>(&point[0]),
                     n, ctx.get());
}

// x509.MarshalECPrivateKey: version 1, d padded to the order's length,
// [0] named curve, [1] the public point.
std::string ec_pem(const Key& k) {
  size_t olen;
  Bytes point;
  ec_public(k, olen, point);
  Bytes d = bn_bytes(k.ec_d.get());
  if (d.size() < olen) d.insert(d.begin(), olen - d.size(), '\0');
  Bytes body = der_small_int(1) + der_tlv(0x04, d) + der_tlv(0xa0, der_oid(k.curve->oid)) +
               der_tlv(0xa1, der_tlv(0x03, Bytes(1, '\0') + point));
  return pem_encode("EC PRIVATE KEY", der_tlv(0x30, body));
}

// x509.ParsePKCS1PrivateKey (two primes; the stored CRT values are ignored).
Key parse_pkcs1(const Bytes& der) {
  Der top(der);
  Der s = top.enter(0x30);
  if (!top.done()) fail("asn1: syntax error: trailing data");
  int64_t version = s.small_int();
  Key k;
  bool neg[5] = {false, false, false, false, false};
  k.n = s.integer(&neg[0]);
  k.e = s.integer(&neg[1]);
  k.d = s.integer(&neg[2]);
  k.p = s.integer(&neg[3]);
  k.q = s.integer(&neg[4]);
  s.integer();
  s.integer();
  s.integer();
  if (version > 1) fail("x509: unsupported private key version");
  if (!s.done()) fail("x509: multi-prime RSA keys are not supported");
  if (neg[0] || neg[2] || neg[3] || neg[4] || BN_is_zero(k.n.get()) || BN_is_zero(k.d.get()) ||
      BN_is_zero(k.p.get()) || BN_is_zero(k.q.get()))
    fail("x509: private key contains zero or negative value");
  if (neg[1]) fail("crypto/rsa: public exponent too small");
  rsa_validate(k);
  k.kind = Key::RSA;
  return k;
}

const Curve* curve_by_oid(const std::string& oid) {
  for (const Curve& c : kCurves)
    if (oid == c.oid) return &c;
  return nullptr;
}

// x509.parseECPrivateKey (SEC1), the curve given by PKCS#8 or by the key.
Key parse_sec1(const Bytes& der, const Curve* named) {
  Der top(der);
  Der s = top.enter(0x30);
  int64_t version = s.small_int();
  Bytes priv = s.raw(0x04);
  std::string oid;
  if (s.peek_tag() == 0xa0) {
    Der p = s.enter(0xa0);
    oid = p.oid();
  }
  if (version != 1) fail("x509: unknown EC private key version " + std::to_string(version));
  const Curve* c = named ? named : curve_by_oid(oid);
  if (!c) fail("x509: unknown elliptic curve");
  Key k;
  k.curve = c;
  k.ec_d = bn_bin(priv);
  std::unique_ptr<EC_GROUP, GroupFree> g(EC_GROUP_new_by_curve_name(c->nid));
  Bn order = bn_new();
  EC_GROUP_get_order(g.get(), order.get(), nullptr);
  if (BN_cmp(k.ec_d.get(), order.get()) >= 0) fail("x509: invalid elliptic curve private key value");
  size_t olen = static_cast<size_t>((BN_num_bits(order.get()) + 7) / 8);
  size_t lead = 0;
  while (priv.size() - lead > olen) {
    if (priv[lead] != 0) fail("x509: invalid private key length");
    lead++;
  }
  k.kind = Key::EC;
  return k;
}

// x509.ParsePKCS8PrivateKey.
Key parse_pkcs8(const Bytes& der) {
  Der top(der);
  Der s = top.enter(0x30);
  s.small_int();
  Der alg = s.enter(0x30);
  std::string oid = alg.oid();
  Bytes inner = s.raw(0x04);
  if (oid == "1.2.840.113549.1.1.1") {
    try {
      return parse_pkcs1(inner);
    } catch (GoError& e) {
      fail("x509: failed to parse RSA private key embedded in PKCS#8: " + e.msg);
    }
  }
  if (oid == "1.2.840.10045.2.1") {
    const Curve* c = nullptr;
    if (!alg.done() && alg.peek_tag() == 0x06) c = curve_by_oid(alg.oid());
    if (!c) fail("x509: unknown elliptic curve");
    try {
      return parse_sec1(inner, c);
    } catch (GoError& e) {
      fail("x509: failed to parse EC private key embedded in PKCS#8: " + e.msg);
    }
  }
  if (oid == "1.3.101.112") {
    Key k;
    k.go_type = "ed25519.PrivateKey";
    return k;
  }
  fail("x509: PKCS#8 wrapping contained private key with unknown algorithm: " + oid);
}

// ssh.ParseDSAPrivateKey: version, p, q, g, y, x.
Key parse_dsa(const Bytes& der) {
  try {
    Der top(der);
    Der s = top.enter(0x30);
    s.small_int();
    for (int i = 0; i < 5; i++) s.integer();
  } catch (GoError& e) {
    fail("ssh: failed to parse DSA key: " + e.msg);
  }
  Key k;
  k.go_type = "*dsa.PrivateKey";
  return k;
}

// ---------------------------------------------------------------------------
// Symmetric ciphers (libcrypto EVP), digests
// ---------------------------------------------------------------------------

Bytes md5(const Bytes& in) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  EVP_Digest(in.data(), in.size(), out, &n, EVP_md5(), nullptr);
  return Bytes(reinterpret_cast<char*>(out), n);
}

Bytes sha512(const Bytes& in) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  EVP_Digest(in.data(), in.size(), out, &n, EVP_sha512(), nullptr);
  return Bytes(reinterpret_cast<char*>(out), n);
}

// Raw block-cipher decryption (no padding handling): CBC or CTR.
Bytes evp_crypt(const EVP_CIPHER* c, const Bytes& key, const Bytes& iv, const Bytes& in) {
  std::unique_ptr<EVP_CIPHER_CTX, CipherCtxFree> ctx(EVP_CIPHER_CTX_new());
  if (!c || !ctx) fail("cipher unavailable");
  if (EVP_DecryptInit_ex(ctx.get(), c, nullptr, reinterpret_cast<const unsigned char*>(key.data()),
                         reinterpret_cast<const unsigned char*>(iv.data())) != 1)
    fail("cipher init failed");
  EVP_CIPHER_CTX_set_padding(ctx.get(), 0);
  Bytes out(in.size() + 32, '\0');
  int n1 = 0, n2 = 0;
  if (EVP_DecryptUpdate(ctx.get(), reinterpret_cast<unsigned char*>(&out[0]), &n1,
                        reinterpret_cast<const unsigned char*>(in.data()), static_cast<int>(in.size())) != 1 ||
      EVP_DecryptFinal_ex(ctx.get(), reinterpret_cast<unsigned char*>(&out[0]) + n1, &n2) != 1)
    fail("cipher failed");
  out.resize(static_cast<size_t>(n1 + n2));
  return out;
}

// ---------------------------------------------------------------------------
// Blowfish and bcrypt_pbkdf (x/crypto/blowfish, x/crypto/ssh/internal/bcrypt_pbkdf)
// ---------------------------------------------------------------------------

struct Blowfish {
  uint32_t p[18];
  uint32_t s[4][256];

  Blowfish() {
    std::memcpy(p, kBlowfishPi, sizeof p);
    std::memcpy(s, kBlowfishPi + 18, sizeof s);
  }

  inline uint32_t f(uint32_t x) const {
    return ((s[0][x >> 24] + s[1][(x >> 16) & 0xff]) ^ s[2][(x >> 8) & 0xff]) + s[3][x & 0xff];
  }

  inline void encrypt(uint32_t& l, uint32_t& r) const {
    uint32_t xl = l ^ p[0], xr = r;
    for (int i = 1; i <= 16; i += 2) {
      xr ^= f(xl) ^ p[i];
      xl ^= f(xr) ^ p[i + 1];
    }
    xr ^= p[17];
    l = xr;
    r = xl;
  }

  static uint32_t next_word(const Bytes& b, size_t& j) {
    uint32_t w = 0;
    for (int k = 0; k < 4; k++) {
      w = (w << 8) | static_cast<unsigned char>(b[j]);
      if (++j >= b.size()) j = 0;
    }
    return w;
  }

  // expandKeyWithSalt (salt non-empty) / ExpandKey (salt empty)
  void expand(const Bytes& key, const Bytes* salt) {
    size_t j = 0;
    for (uint32_t& w : p) w ^= next_word(key, j);
    j = 0;
    uint32_t l = 0, r = 0;
    auto step = [&](uint32_t& a, uint32_t& b) {
      if (salt) {
        l ^= next_word(*salt, j);
        r ^= next_word(*salt, j);
      }
      encrypt(l, r);
      a = l;
      b = r;
    };
    for (int i = 0; i < 18; i += 2) step(p[i], p[i + 1]);
    for (auto& box : s)
      for (int i = 0; i < 256; i += 2) step(box[i], box[i + 1]);
  }
};

void bcrypt_hash(uint8_t out[32], const Bytes& shapass, const Bytes& shasalt) {
  Blowfish c;
  c.expand(shapass, &shasalt);
  for (int i = 0; i < 64; i++) {
    c.expand(shasalt, nullptr);
    c.expand(shapass, nullptr);
  }
  static const char magic[] = "OxychromaticBlowfishSwatDynamite";
  uint32_t w[8];
  for (int i = 0; i < 8; i++)
    w[i] = (static_cast<uint32_t>(static_cast<unsigned char>(magic[4 * i])) << 24) |
           (static_cast<uint32_t>(static_cast<unsigned char>(magic[4 * i + 1])) << 16) |
           (static_cast<uint32_t>(static_cast<unsigned char>(magic[4 * i + 2])) << 8) |
           static_cast<uint32_t>(static_cast<unsigned char>(magic[4 * i + 3]));
  for (int b = 0; b < 8; b += 2)
    for (int k = 0; k < 64; k++) c.encrypt(w[b], w[b + 1]);
  for (int i = 0; i < 8; i++) {  // little-endian words out
    out[4 * i] = static_cast<uint8_t>(w[i]);
    out[4 * i + 1] = static_cast<uint8_t>(w[i] >> 8);
    out[4 * i + 2] = static_cast<uint8_t>(w[i] >> 16);
    out[4 * i + 3] = static_cast<uint8_t>(w[i] >> 24);
  }
}

constexpr uint32_t kMaxBcryptRounds = 4096;

Bytes bcrypt_pbkdf(const Bytes& password, const Bytes& salt, int64_t rounds, int64_t key_len) {
  if (rounds < 1) fail("bcrypt_pbkdf: number of rounds is too small");
  if (password.empty()) fail("bcrypt_pbkdf: empty password");
  if (salt.empty() || salt.size() > (1u << 20)) fail("bcrypt_pbkdf: bad salt length");
  if (key_len > 1024) fail("bcrypt_pbkdf: keyLen is too large");
  const int64_t block = 32;
  int64_t nblocks = (key_len + block - 1) / block;
  Bytes key(static_cast<size_t>(nblocks * block), '\0');
  Bytes shapass = sha512(password);
  uint8_t tmp[32], out[32];
  for (int64_t b = 1; b <= nblocks; b++) {
    Bytes cs = salt;
    cs += static_cast<char>(b >> 24);
    cs += static_cast<char>(b >> 16);
    cs += static_cast<char>(b >> 8);
    cs += static_cast<char>(b);
    bcrypt_hash(tmp, shapass, sha512(cs));
    std::memcpy(out, tmp, 32);
    for (int64_t r = 2; r <= rounds; r++) {
      bcrypt_hash(tmp, shapass, sha512(Bytes(reinterpret_cast<char*>(tmp), 32)));
      for (int j = 0; j < 32; j++) out[j] ^= tmp[j];
    }
    for (int i = 0; i < 32; i++) key[static_cast<size_t>(i * nblocks + (b - 1))] = static_cast<char>(out[i]);
  }
  key.resize(static_cast<size_t>(key_len));
  return key;
}

// ---------------------------------------------------------------------------
// openssh-key-v1 (x/crypto/ssh keys.go parseOpenSSHPrivateKey)
// ---------------------------------------------------------------------------

struct Wire {
  const Bytes& b;
  size_t i = 0;
  explicit Wire(const Bytes& buf) : b(buf) {}
  uint32_t u32() {
    if (i + 4 > b.size()) fail("ssh: short read");
    uint32_t v = (static_cast<uint32_t>(static_cast<unsigned char>(b[i])) << 24) |
                 (static_cast<uint32_t>(static_cast<unsigned char>(b[i + 1])) << 16) |
                 (static_cast<uint32_t>(static_cast<unsigned char>(b[i + 2])) << 8) |
                 static_cast<uint32_t>(static_cast<unsigned char>(b[i + 3]));
    i += 4;
    return v;
  }
  Bytes str() {
    uint32_t n = u32();
    if (i + n > b.size()) fail("ssh: short read");
    Bytes s = b.substr(i, n);
    i += n;
    return s;
  }
  Bn mpint(bool* negative = nullptr) {
    Bytes s = str();
    bool neg = !s.empty() && (s[0] & 0x80);
    if (negative) *negative = neg;
    return neg ? bn_new() : bn_bin(s);
  }
  Bytes rest() { return b.substr(i); }
};

void check_padding(const Bytes& pad) {
  for (size_t k = 0; k < pad.size(); k++)
    if (static_cast<unsigned char>(pad[k]) != ((k + 1) & 0xff)) fail("ssh: padding not as expected");
}

const char kIncorrectPassword[] = "x509: decryption password incorrect";

Key parse_openssh(const Bytes& data, const Bytes* passphrase) {
  static const Bytes magic("openssh-key-v1\0", 15);
  if (data.size() < magic.size() || data.compare(0, magic.size(), magic) != 0)
    fail("ssh: invalid openssh private key format");
  Bytes body = data.substr(magic.size());
  Wire w(body);
  Bytes cipher = w.str(), kdf = w.str(), kdfopts = w.str();
  uint32_t nkeys = w.u32();
  w.str();  // public key
  Bytes block = w.str();
  if (nkeys != 1) fail("ssh: multi-key files are not supported");
  if (!passphrase) {
    if (kdf != "none" || cipher != "none") throw PassphraseMissing();
    if (!kdfopts.empty()) fail("ssh: invalid openssh private key");
  } else {
    if (kdf == "none" || cipher == "none") fail("ssh: key is not password protected");
    if (kdf != "bcrypt") fail("ssh: unknown KDF " + go_quote(kdf) + ", only supports \"bcrypt\"");
    Wire o(kdfopts);
    Bytes salt = o.str();
    uint32_t rounds = o.u32();
    // x/crypto/ssh passes any count to bcrypt_pbkdf: a file asking for 2^32
    // rounds makes the reference (and ssh-keygen) spin for days; refused here
    // (DEVIATIONS.md 6).  ssh-keygen writes 16 unless told otherwise (-a).
    if (rounds > kMaxBcryptRounds)
      fail("ssh: bcrypt_pbkdf rounds " + std::to_string(rounds) + " exceed the limit of " +
           std::to_string(kMaxBcryptRounds));
    Bytes k = bcrypt_pbkdf(*passphrase, salt, rounds, 32 + 16);
    Bytes key = k.substr(0, 32), iv = k.substr(32);
    if (cipher == "aes256-ctr") {
      block = evp_crypt(EVP_aes_256_ctr(), key, iv, block);
    } else if (cipher == "aes256-cbc") {
      if (block.size() % 16 != 0)
        fail("ssh: invalid encrypted private key length, not a multiple of the block size");
      block = evp_crypt(EVP_aes_256_cbc(), key, iv, block);
    } else {
      fail("ssh: unknown cipher " + go_quote(cipher) + ", only supports \"aes256-ctr\" or \"aes256-cbc\"");
    }
  }
  Wire pk(block);
  uint32_t c1, c2;
  Bytes keytype;
  try {
    c1 = pk.u32();
    c2 = pk.u32();
    keytype = pk.str();
  } catch (GoError&) {
    c1 = 0;
    c2 = 1;
  }
  if (c1 != c2) {
    if (cipher != "none") fail(kIncorrectPassword);
    fail("ssh: malformed OpenSSH key");
  }
  Key k;
  if (keytype == "ssh-rsa") {
    bool neg_e = false;
    k.n = pk.mpint();
    k.e = pk.mpint(&neg_e);
    k.d = pk.mpint();
    pk.mpint();  // iqmp: recomputed by Precompute
    k.p = pk.mpint();
    k.q = pk.mpint();
    pk.str();  // comment
    check_padding(pk.rest());
    if (neg_e) fail("crypto/rsa: public exponent too small");
    rsa_validate(k);
    k.kind = Key::RSA;
    return k;
  }
  if (keytype == "ssh-ed25519") {
    pk.str();
    Bytes priv = pk.str();
    pk.str();
    check_padding(pk.rest());
    if (priv.size() != 64) fail("ssh: private key unexpected length");
    k.go_type = "*ed25519.PrivateKey";
    return k;
  }
  if (keytype.compare(0, 11, "ecdsa-sha2-") == 0) {
    Bytes curve_name = pk.str();
    Bytes pub = pk.str();
    k.ec_d = pk.mpint();
    pk.str();
    check_padding(pk.rest());
    for (const Curve& c : kCurves)
      if (curve_name == c.ssh_name && *c.ssh_name) k.curve = &c;
    if (!k.curve) fail("ssh: unhandled elliptic curve: " + curve_name);
    std::unique_ptr<EC_GROUP, GroupFree> g(EC_GROUP_new_by_curve_name(k.curve->nid));
    std::unique_ptr<BN_CTX, CtxFree> ctx(BN_CTX_new());
    std::unique_ptr<EC_POINT, PointFree> q(EC_POINT_new(g.get()));
    if (pub.empty() || pub[0] != 4 ||
        !EC_POINT_oct2point(g.get(), q.get(), reinterpret_cast<const unsigned char*>(pub.data()), pub.size(),
                            ctx.get()))
      fail("ssh: failed to unmarshal public key");
    Bn order = bn_new();
    EC_GROUP_get_order(g.get(), order.get(), ctx.get());
    if (BN_cmp(k.ec_d.get(), order.get()) >= 0) fail("ssh: scalar is out of range");
    size_t olen;
    Bytes point;
    ec_public(k, olen, point);
    if (point != pub) fail("ssh: public key does not match private key");
    k.kind = Key::EC;
    return k;
  }
  fail("ssh: unhandled key type");
}

// ---------------------------------------------------------------------------
// Legacy encrypted PEM (x509.DecryptPEMBlock)
// ---------------------------------------------------------------------------

Bytes decrypt_pem_block(const PemBlock& blk, const Bytes& password) {
  const std::string* dek = blk.header("DEK-Info");
  if (!dek) fail("x509: no DEK-Info header in block");
  size_t comma = dek->find(',');
  if (comma == std::string::npos) fail("x509: malformed DEK-Info header");
  std::string mode = dek->substr(0, comma), hexiv = dek->substr(comma + 1);
  size_t key_size, block_size = 16;
  const EVP_CIPHER* c = nullptr;
  bool single_des = false;
  if (mode == "DES-CBC") {
    key_size = 8;
    block_size = 8;
    single_des = true;
    c = EVP_des_ede3_cbc();  // DES-EDE3 with K1 = K2 = K3 is single DES
  } else if (mode == "DES-EDE3-CBC") {
    key_size = 24;
    block_size = 8;
    c = EVP_des_ede3_cbc();
  } else if (mode == "AES-128-CBC") {
    key_size = 16;
    c = EVP_aes_128_cbc();
  } else if (mode == "AES-192-CBC") {
    key_size = 24;
    c = EVP_aes_192_cbc();
  } else if (mode == "AES-256-CBC") {
    key_size = 32;
    c = EVP_aes_256_cbc();
  } else {
    fail("x509: unknown encryption mode");
  }
  if (hexiv.size() % 2) fail("encoding/hex: odd length hex string");
  Bytes iv;
  for (size_t i = 0; i < hexiv.size(); i += 2) {
    auto hv = [&](char ch) -> int {
      if (ch >= '0' && ch <= '9') return ch - '0';
      if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
      if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
      char u[16];
      std::snprintf(u, sizeof u, "U+%04X", static_cast<unsigned char>(ch));
      fail(std::string("encoding/hex: invalid byte: ") + u + " '" + std::string(1, ch) + "'");
    };
    iv += static_cast<char>(hv(hexiv[i]) * 16 + hv(hexiv[i + 1]));
  }
  if (iv.size() != block_size) fail("x509: incorrect IV size");
  // rfc1423Algo.deriveKey: MD5(prev || password || salt[:8]) chained
  Bytes key, digest;
  while (key.size() < key_size) {
    digest = md5(digest + password + iv.substr(0, 8));
    key += digest;
  }
  key.resize(key_size);
  if (single_des) key = key + key + key;
  if (blk.bytes.size() % block_size != 0) fail("x509: encrypted PEM data is not a multiple of the block size");
  Bytes data = evp_crypt(c, key, iv, blk.bytes);
  size_t dlen = data.size();
  if (dlen == 0 || dlen % block_size != 0) fail("x509: invalid padding");
  size_t last = static_cast<unsigned char>(data[dlen - 1]);
  if (dlen < last || last == 0 || last > block_size) fail(kIncorrectPassword);
  for (size_t k = dlen - last; k < dlen; k++)
    if (static_cast<unsigned char>(data[k]) != last) fail(kIncorrectPassword);
  data.resize(dlen - last);
  return data;
}

// ---------------------------------------------------------------------------
// ssh.ParseRawPrivateKey / ParseRawPrivateKeyWithPassphrase
// ---------------------------------------------------------------------------

bool encrypted_block(const PemBlock& b) {
  const std::string* pt = b.header("Proc-Type");
  return pt && pt->find("ENCRYPTED") != std::string::npos;
}

Key parse_raw(const Bytes& data, const Bytes* passphrase) {
  PemBlock blk;
  if (!pem_decode(data, blk)) fail("ssh: no key found");
  if (!passphrase) {
    if (encrypted_block(blk)) throw PassphraseMissing();
    if (blk.type == "RSA PRIVATE KEY") return parse_pkcs1(blk.bytes);
    if (blk.type == "PRIVATE KEY") return parse_pkcs8(blk.bytes);
    if (blk.type == "EC PRIVATE KEY") return parse_sec1(blk.bytes, nullptr);
    if (blk.type == "DSA PRIVATE KEY") return parse_dsa(blk.bytes);
    if (blk.type == "OPENSSH PRIVATE KEY") return parse_openssh(blk.bytes, nullptr);
    fail("ssh: unsupported key type " + go_quote(blk.type));
  }
  if (blk.type == "OPENSSH PRIVATE KEY") return parse_openssh(blk.bytes, passphrase);
  if (!encrypted_block(blk) || !blk.header("DEK-Info")) fail("ssh: not an encrypted key");
  Bytes buf;
  try {
    buf = decrypt_pem_block(blk, *passphrase);
  } catch (GoError& e) {
    if (e.msg == kIncorrectPassword) throw;
    fail("ssh: cannot decode encrypted private keys: " + e.msg);
  }
  if (blk.type == "RSA PRIVATE KEY") return parse_pkcs1(buf);
  if (blk.type == "EC PRIVATE KEY") return parse_sec1(buf, nullptr);
  if (blk.type == "DSA PRIVATE KEY") return parse_dsa(buf);
  fail("ssh: unsupported key type " + go_quote(blk.type));
}

// (status, text): 0 the PEM, 1 passphrase missing, 2 an error, 3 an
// unsupported key type (its Go %T).
// A Go string as Python text: error messages can carry bytes of the key
// file, which need not be UTF-8; they survive as surrogate escapes (the
// caller's %q prints them as \xNN, as Go's does).
py::str go_text(const std::string& s) {
  PyObject* o = PyUnicode_DecodeUTF8(s.data(), (Py_ssize_t)s.size(), "surrogateescape");
  if (!o) throw py::error_already_set();
  return py::reinterpret_steal<py::str>(o);
}

py::tuple private_key_pem(py::bytes data, py::object passphrase) {
  Bytes in = data;
  Bytes pass;
  bool has_pass = !passphrase.is_none();
  if (has_pass) pass = passphrase.cast<py::bytes>();
  int status;
  std::string text;
  {
    py::gil_scoped_release nogil;
    try {
      Key k = parse_raw(in, has_pass ? &pass : nullptr);
      if (k.kind == Key::RSA) {
        status = 0;
        text = rsa_pem(k);
      } else if (k.kind == Key::EC) {
        status = 0;
        text = ec_pem(k);
      } else {
        status = 3;
        text = k.go_type;
      }
    } catch (PassphraseMissing&) {
      status = 1;
      text = "ssh: this private key is passphrase protected";
    } catch (GoError& e) {
      status = 2;
      text = e.msg;
    }
  }
  OPENSSL_cleanse(&pass[0], pass.size());
  return py::make_tuple(status, go_text(text));
}

py::bytes py_bcrypt_pbkdf(py::bytes password, py::bytes salt, int64_t rounds, int64_t key_len) {
  try {
    return py::bytes(bcrypt_pbkdf(password, salt, rounds, key_len));
  } catch (GoError& e) {
    throw py::value_error(e.msg);
  }
}

py::object py_pem_decode(py::bytes data) {
  PemBlock b;
  if (!pem_decode(data, b)) return py::none();
  py::list headers;
  for (auto& h : b.headers) headers.append(py::make_tuple(go_text(h.first), go_text(h.second)));
  return py::make_tuple(go_text(b.type), headers, py::bytes(b.bytes));
}

}  // namespace

PYBIND11_MODULE(_m2k_sshkey, m) {
  m.doc() = "private SSH keys parsed, decrypted and re-encoded as PEM in process (sshkeys.go:170-232)";
  m.def("private_key_pem", &private_key_pem, py::arg("data"), py::arg("passphrase") = py::none());
  m.def("bcrypt_pbkdf", &py_bcrypt_pbkdf, py::arg("password"), py::arg("salt"), py::arg("rounds"),
        py::arg("key_len"));
  m.def("pem_decode", &py_pem_decode, py::arg("data"));
}
