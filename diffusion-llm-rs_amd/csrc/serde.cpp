// serde.cpp -- wire formats of the quantized objects behind the C-ABI, for a
// Rust or C++ caller that checkpoints or hands off quantized tensors without the Python package.
//
// Objects (the reference's #[derive(Serialize, Deserialize)] structs):
//   QuantizationParams {bits: u8, scale: f32, zero_point: i32, symmetric: bool, axis: Option<usize>}
//     and QuantizedTensor {data: Vec<u8>, shape: Vec<usize>, params}  (quantization/src/types.rs:19-47)
//   CompressedVector {id: String, data: Vec<u8>, bits: u8, original_shape: Vec<usize>,
//     quant_scale: f32, quant_zero_point: f32}                        (diffusion_prefill/src/prefill_kv.rs:25-33)
// Encodings, restated from their published specifications (the crates are absent from the image):
//   bincode 1.3 legacy `serialize`: little-endian fixed-width integers, usize as u64, Vec/String =
//     u64 length + elements, bool 1 byte, Option = 1-byte tag (+ value).  `deserialize` (the legacy
//     free function) ignores trailing bytes; strict = 1 rejects them (DefaultOptions).
//   serde_json `to_string`: compact, fields in declaration order, Vec<u8> as an integer array, None as
//     null, f32 as ryu's shortest round-trip digits in ryu's layout, non-finite f32 as null.
// The same layouts as diffusion-llm-rs_amd/serde.py; tests/test_serde_capi.py checks the two agree
// byte for byte and round-trips both directions.
#include <cerrno>
#include <charconv>
#include <climits>
#include <cmath>
#include <cstring>
#include <string>
#include <initializer_list>
#include <vector>

#include "common.hpp"

namespace dllm {
namespace {

struct Writer {
    std::string b;
    void u8(uint8_t v) { b.push_back(static_cast<char>(v)); }
    void raw(const void *p, size_t n) { b.append(static_cast<const char *>(p), n); }
    void u64(uint64_t v) { raw(&v, 8); }   // x86-64 and gfx950 hosts are little-endian
    void i32(int32_t v) { raw(&v, 4); }
    void f32(float v) { raw(&v, 4); }
    void bytes(const uint8_t *p, size_t n) { u64(n); raw(p, n); }
    void usizes(const uint64_t *p, size_t n) {
        u64(n);
        for (size_t i = 0; i < n; ++i) u64(p[i]);
    }
};

struct Reader {
    const uint8_t *p;
    size_t n, i = 0;
    bool ok = true;
    bool take(void *dst, size_t k) {
        if (!ok || i + k > n || i + k < i) return ok = false;
        std::memcpy(dst, p + i, k);
        i += k;
        return true;
    }
    uint8_t u8() { uint8_t v = 0; take(&v, 1); return v; }
    uint64_t u64() { uint64_t v = 0; take(&v, 8); return v; }
    int32_t i32() { int32_t v = 0; take(&v, 4); return v; }
    float f32() { float v = 0; take(&v, 4); return v; }
};

void put_params(Writer &w, const dllm_qparams *p) {
    w.u8(p->bits);
    w.f32(p->scale);
    w.i32(p->zero_point);
    w.u8(p->symmetric ? 1 : 0);
    if (p->has_axis) {
        w.u8(1);
        w.u64(p->axis);
    } else {
        w.u8(0);
    }
}

int get_params(Reader &r, dllm_qparams *p) {
    p->bits = r.u8();
    p->scale = r.f32();
    p->zero_point = r.i32();
    const uint8_t sym = r.u8(), tag = r.u8();
    if (!r.ok) return fail(DLLM_ERR_SERIALIZATION, "bincode: unexpected end of input");
    if (sym > 1) return fail(DLLM_ERR_SERIALIZATION, "bincode: invalid bool");
    if (tag > 1) return fail(DLLM_ERR_SERIALIZATION, "bincode: invalid Option tag");
    p->symmetric = sym;
    p->has_axis = tag;
    p->axis = tag ? r.u64() : 0;
    if (!r.ok) return fail(DLLM_ERR_SERIALIZATION, "bincode: unexpected end of input");
    return DLLM_OK;
}

int emit(const std::string &s, void *out, size_t cap, size_t *len) {
    if (len) *len = s.size();
    if (!out) return DLLM_OK;   // size query
    if (cap < s.size()) return fail(DLLM_ERR_SERIALIZATION, "output buffer too small (see *len)");
    std::memcpy(out, s.data(), s.size());
    return DLLM_OK;
}

int finish(const Reader &r, int strict, size_t *consumed) {
    if (consumed) *consumed = r.i;
    if (strict && r.i != r.n) return fail(DLLM_ERR_SERIALIZATION, "bincode: trailing bytes");
    return DLLM_OK;
}

// ryu::Buffer::format_finite(f32) (ryu/src/pretty/mod.rs format32): shortest round-trip digits,
// laid out plain for 10^-5 <= |x| < 10^13 (kk in (-6, 13]) and as d.ddde<exp> otherwise.
std::string ryu_f32(float x) {
    uint32_t bits;
    std::memcpy(&bits, &x, 4);
    const std::string sign = (bits >> 31) ? "-" : "";
    if ((bits & 0x7FFFFFFFu) == 0) return sign + "0.0";
    char buf[64];
    const auto res = std::to_chars(buf, buf + sizeof(buf), std::fabs(x), std::chars_format::scientific);
    const std::string sci(buf, res.ptr);
    const size_t epos = sci.find('e');
    std::string mant = sci.substr(0, epos);
    const int e10 = std::stoi(sci.substr(epos + 1));
    std::string digits;
    for (char c : mant)
        if (c != '.') digits.push_back(c);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const int length = static_cast<int>(digits.size());
    const int k = e10 - (length - 1), kk = length + k;
    std::string out;
    if (0 <= k && kk <= 13) {
        out = digits + std::string(static_cast<size_t>(kk - length), '0') + ".0";
    } else if (0 < kk && kk <= 13) {
        out = digits.substr(0, static_cast<size_t>(kk)) + "." + digits.substr(static_cast<size_t>(kk));
    } else if (-6 < kk && kk <= 0) {
        out = "0." + std::string(static_cast<size_t>(-kk), '0') + digits;
    } else if (length == 1) {
        out = digits + "e" + std::to_string(kk - 1);
    } else {
        out = digits.substr(0, 1) + "." + digits.substr(1) + "e" + std::to_string(kk - 1);
    }
    return sign + out;
}

std::string json_f32(float x) { return std::isfinite(x) ? ryu_f32(x) : "null"; }

std::string json_u8s(const uint8_t *p, size_t n) {
    std::string s = "[";
    for (size_t i = 0; i < n; ++i) {
        if (i) s.push_back(',');
        s += std::to_string(static_cast<unsigned>(p[i]));
    }
    return s + "]";
}

std::string json_usizes(const uint64_t *p, size_t n) {
    std::string s = "[";
    for (size_t i = 0; i < n; ++i) {
        if (i) s.push_back(',');
        s += std::to_string(static_cast<unsigned long long>(p[i]));
    }
    return s + "]";
}

std::string json_params(const dllm_qparams *p) {
    return "{\"bits\":" + std::to_string(static_cast<unsigned>(p->bits)) + ",\"scale\":" + json_f32(p->scale) +
           ",\"zero_point\":" + std::to_string(p->zero_point) + ",\"symmetric\":" + (p->symmetric ? "true" : "false") +
           ",\"axis\":" + (p->has_axis ? std::to_string(static_cast<unsigned long long>(p->axis)) : "null") + "}";
}

// serde_json string escaping (its `format_escaped_str`): ", \ and control characters.
std::string json_str(const char *s, size_t n) {
    static const char *hex = "0123456789abcdef";
    std::string o = "\"";
    for (size_t i = 0; i < n; ++i) {
        const unsigned char c = static_cast<unsigned char>(s[i]);
        switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\b': o += "\\b"; break;
        case '\f': o += "\\f"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        default:
            if (c < 0x20) {
                o += "\\u00";
                o.push_back(hex[c >> 4]);
                o.push_back(hex[c & 15]);
            } else {
                o.push_back(static_cast<char>(c));
            }
        }
    }
    return o + "\"";
}

// Length of the valid UTF-8 sequence at u[0 .. n) (RFC 3629: no overlong forms, no surrogates,
// at most U+10FFFF), or 0 when it is not one.
size_t utf8_len(const unsigned char *u, size_t n) {
    const unsigned c = u[0];
    if (c < 0x80) return 1;
    const size_t k = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (!k || k > n) return 0;
    unsigned cp = c & (0x7F >> k);
    for (size_t j = 1; j < k; ++j) {
        if ((u[j] >> 6) != 2) return 0;
        cp = (cp << 6) | (u[j] & 63);
    }
    static const unsigned lo[5] = {0, 0, 0x80, 0x800, 0x10000};
    if (cp < lo[k] || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return 0;
    return k;
}

// ---- minimal JSON reader for the fixed schemas (serde_json's compact and pretty output) ----------
// Field handling follows serde's derived Deserialize: unknown fields are skipped, a repeated field
// is an error ("duplicate field"), a missing one too.
struct JReader {
    const char *p, *e;
    bool ok = true;
    void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p; }
    bool lit(const char *s) {
        ws();
        const size_t n = std::strlen(s);
        if (static_cast<size_t>(e - p) >= n && std::strncmp(p, s, n) == 0) { p += n; return true; }
        return false;
    }
    void expect(char c) { if (!lit(std::string(1, c).c_str())) ok = false; }
    std::string key() {
        std::string k;
        if (!string(k)) return {};
        expect(':');
        return k;
    }
    // Skips one value of any type: the value of a field the schema does not name (serde's derived
    // Deserialize ignores unknown fields unless deny_unknown_fields).
    bool skip_value(int depth = 0) {
        ws();
        if (p >= e || depth > 128) return ok = false;
        if (*p == '"') { std::string t; return string(t); }
        if (*p == '{' || *p == '[') {
            const char close = *p == '{' ? '}' : ']';
            const bool obj = *p == '{';
            ++p;
            if (lit(std::string(1, close).c_str())) return true;
            do {
                if (obj) { key(); if (!ok) return false; }
                if (!skip_value(depth + 1)) return false;
            } while (lit(","));
            expect(close);
            return ok;
        }
        if (lit("true") || lit("false") || lit("null")) return true;
        number();
        return ok;
    }
    bool null() { return lit("null"); }
    // a JSON number as f64 (serde parses f32 fields through f64 and rounds: f32 visitor)
    double number() {
        ws();
        const char *s = p;
        while (p < e && (std::strchr("+-0123456789.eE", *p) != nullptr)) ++p;
        if (s == p) { ok = false; return 0; }
        return std::strtod(std::string(s, p).c_str(), nullptr);
    }
    bool integer(long long lo, long long hi, long long &v) {
        ws();
        const char *s = p;
        if (p < e && *p == '-') ++p;
        while (p < e && *p >= '0' && *p <= '9') ++p;
        if (s == p || (p < e && (*p == '.' || *p == 'e' || *p == 'E'))) { ok = false; return false; }
        errno = 0;
        v = std::strtoll(std::string(s, p).c_str(), nullptr, 10);
        if (errno || v < lo || v > hi) { ok = false; return false; }
        return true;
    }
    template <typename T>
    bool int_array(long long lo, long long hi, std::vector<T> &out) {
        expect('[');
        if (lit("]")) return ok;
        do {
            long long v;
            if (!integer(lo, hi, v)) return false;
            out.push_back(static_cast<T>(v));
        } while (lit(","));
        expect(']');
        return ok;
    }
    bool boolean(uint8_t &v) {
        if (lit("true")) { v = 1; return true; }
        if (lit("false")) { v = 0; return true; }
        return ok = false;
    }
    float f32_or_null() { return null() ? NAN : static_cast<float>(number()); }
    // a JSON string value as UTF-8 (serde_json's string reader: the escapes of RFC 8259 including
    // \uXXXX surrogate pairs; raw control characters and lone surrogates are errors)
    bool hex4(unsigned &v) {
        if (e - p < 4) return false;
        v = 0;
        for (int i = 0; i < 4; ++i) {
            const char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else return false;
        }
        return true;
    }
    static void utf8(std::string &o, unsigned cp) {
        if (cp < 0x80) {
            o.push_back(static_cast<char>(cp));
        } else if (cp < 0x800) {
            o.push_back(static_cast<char>(0xC0 | (cp >> 6)));
            o.push_back(static_cast<char>(0x80 | (cp & 63)));
        } else if (cp < 0x10000) {
            o.push_back(static_cast<char>(0xE0 | (cp >> 12)));
            o.push_back(static_cast<char>(0x80 | ((cp >> 6) & 63)));
            o.push_back(static_cast<char>(0x80 | (cp & 63)));
        } else {
            o.push_back(static_cast<char>(0xF0 | (cp >> 18)));
            o.push_back(static_cast<char>(0x80 | ((cp >> 12) & 63)));
            o.push_back(static_cast<char>(0x80 | ((cp >> 6) & 63)));
            o.push_back(static_cast<char>(0x80 | (cp & 63)));
        }
    }
    bool string(std::string &o) {
        ws();
        if (p >= e || *p != '"') return ok = false;
        ++p;
        while (p < e && *p != '"') {
            const unsigned char c = static_cast<unsigned char>(*p);
            if (c < 0x20) return ok = false;
            if (c >= 0x80) {   // raw UTF-8: the input must be valid UTF-8 (serde_json::from_slice)
                const size_t k = utf8_len(reinterpret_cast<const unsigned char *>(p), static_cast<size_t>(e - p));
                if (!k) return ok = false;
                o.append(p, k);
                p += k;
                continue;
            }
            if (c != '\\') { o.push_back(*p++); continue; }
            if (++p >= e) return ok = false;
            const char x = *p++;
            switch (x) {
            case '"': o.push_back('"'); break;
            case '\\': o.push_back('\\'); break;
            case '/': o.push_back('/'); break;
            case 'b': o.push_back('\b'); break;
            case 'f': o.push_back('\f'); break;
            case 'n': o.push_back('\n'); break;
            case 'r': o.push_back('\r'); break;
            case 't': o.push_back('\t'); break;
            case 'u': {
                unsigned cp;
                if (!hex4(cp)) return ok = false;
                if (cp >= 0xDC00 && cp <= 0xDFFF) return ok = false;
                if (cp >= 0xD800 && cp <= 0xDBFF) {
                    unsigned lo;
                    if (e - p < 6 || p[0] != '\\' || p[1] != 'u') return ok = false;
                    p += 2;
                    if (!hex4(lo) || lo < 0xDC00 || lo > 0xDFFF) return ok = false;
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                }
                utf8(o, cp);
                break;
            }
            default: return ok = false;
            }
        }
        if (p >= e) return ok = false;
        ++p;
        return true;
    }
};

int field_index(const std::string &k, std::initializer_list<const char *> names) {
    int i = 0;
    for (const char *n : names) {
        if (k == n) return i;
        ++i;
    }
    return -1;
}

int parse_params(JReader &j, dllm_qparams *p) {
    j.expect('{');
    bool seen[5] = {false, false, false, false, false};
    if (!j.lit("}")) {
        do {
            const std::string k = j.key();
            long long v;
            const int f = field_index(k, {"bits", "scale", "zero_point", "symmetric", "axis"});
            if (f >= 0 && seen[f]) return fail(DLLM_ERR_SERIALIZATION, "json: duplicate field of QuantizationParams");
            if (f >= 0) seen[f] = true;
            if (f == 0) { if (j.integer(0, 255, v)) p->bits = static_cast<uint8_t>(v); }
            else if (f == 1) { p->scale = j.f32_or_null(); }
            else if (f == 2) { if (j.integer(INT32_MIN, INT32_MAX, v)) p->zero_point = static_cast<int32_t>(v); }
            else if (f == 3) { j.boolean(p->symmetric); }
            else if (f == 4) {
                if (j.null()) { p->has_axis = 0; p->axis = 0; }
                else if (j.integer(0, INT64_MAX, v)) { p->has_axis = 1; p->axis = static_cast<uint64_t>(v); }
            } else {
                j.skip_value();
            }
        } while (j.ok && j.lit(","));
        j.expect('}');
    }
    if (!j.ok) return fail(DLLM_ERR_SERIALIZATION, "json: malformed QuantizationParams");
    for (bool s : seen)
        if (!s) return fail(DLLM_ERR_SERIALIZATION, "json: missing field of QuantizationParams");
    return DLLM_OK;
}

}  // namespace
}  // namespace dllm

using namespace dllm;

extern "C" {

int dllm_format_f32(float x, char *out, size_t cap, size_t *len) { return emit(json_f32(x), out, cap, len); }

int dllm_qparams_to_bincode(const dllm_qparams *p, uint8_t *out, size_t cap, size_t *len) {
    if (!p) return fail(DLLM_ERR_INVALID_PARAMS, "null params");
    Writer w;
    put_params(w, p);
    return emit(w.b, out, cap, len);
}

int dllm_qparams_from_bincode(const uint8_t *buf, size_t len, int strict, dllm_qparams *p, size_t *consumed) {
    if ((!buf && len) || !p) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    Reader r{buf, len};
    if (const int rc = get_params(r, p)) return rc;
    return finish(r, strict, consumed);
}

int dllm_qparams_to_json(const dllm_qparams *p, char *out, size_t cap, size_t *len) {
    if (!p) return fail(DLLM_ERR_INVALID_PARAMS, "null params");
    return emit(json_params(p), out, cap, len);
}

int dllm_qparams_from_json(const char *s, size_t len, dllm_qparams *p) {
    if ((!s && len) || !p) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    JReader j{s, s + len};
    if (const int rc = parse_params(j, p)) return rc;
    j.ws();
    if (j.p != j.e) return fail(DLLM_ERR_SERIALIZATION, "json: trailing characters");
    return DLLM_OK;
}

int dllm_qtensor_to_bincode(const uint8_t *codes, size_t n, const uint64_t *shape, size_t ndim, const dllm_qparams *p,
                            uint8_t *out, size_t cap, size_t *len) {
    if ((!codes && n) || (!shape && ndim) || !p) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    Writer w;
    w.bytes(codes, n);
    w.usizes(shape, ndim);
    put_params(w, p);
    return emit(w.b, out, cap, len);
}

int dllm_qtensor_from_bincode(const uint8_t *buf, size_t len, int strict, uint8_t *codes, size_t codes_cap, size_t *n,
                              uint64_t *shape, size_t shape_cap, size_t *ndim, dllm_qparams *p) {
    if ((!buf && len) || !n || !ndim || !p) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    Reader r{buf, len};
    const uint64_t nd = r.u64();
    if (!r.ok || nd > len - r.i) return fail(DLLM_ERR_SERIALIZATION, "bincode: unexpected end of input");
    *n = nd;
    if (codes && codes_cap < nd) return fail(DLLM_ERR_INVALID_PARAMS, "codes buffer too small (see *n)");
    if (codes) r.take(codes, nd);
    else r.i += nd;
    const uint64_t ns = r.u64();
    if (!r.ok || ns > (len - r.i) / 8) return fail(DLLM_ERR_SERIALIZATION, "bincode: unexpected end of input");
    *ndim = ns;
    if (shape && shape_cap < ns) return fail(DLLM_ERR_INVALID_PARAMS, "shape buffer too small (see *ndim)");
    for (uint64_t i = 0; i < ns; ++i) {
        const uint64_t v = r.u64();
        if (shape) shape[i] = v;
    }
    if (const int rc = get_params(r, p)) return rc;
    return finish(r, strict, nullptr);
}

int dllm_qtensor_to_json(const uint8_t *codes, size_t n, const uint64_t *shape, size_t ndim, const dllm_qparams *p,
                         char *out, size_t cap, size_t *len) {
    if ((!codes && n) || (!shape && ndim) || !p) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    const std::string s = "{\"data\":" + json_u8s(codes, n) + ",\"shape\":" + json_usizes(shape, ndim) +
                          ",\"params\":" + json_params(p) + "}";
    return emit(s, out, cap, len);
}

int dllm_qtensor_from_json(const char *s, size_t len, uint8_t *codes, size_t codes_cap, size_t *n, uint64_t *shape,
                           size_t shape_cap, size_t *ndim, dllm_qparams *p) {
    if ((!s && len) || !n || !ndim || !p) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    JReader j{s, s + len};
    std::vector<uint8_t> data;
    std::vector<uint64_t> dims;
    bool seen[3] = {false, false, false};
    j.expect('{');
    if (!j.lit("}")) {
        do {
            const std::string k = j.key();
            const int f = field_index(k, {"data", "shape", "params"});
            if (f >= 0 && seen[f]) return fail(DLLM_ERR_SERIALIZATION, "json: duplicate field of QuantizedTensor");
            if (f >= 0) seen[f] = true;
            if (f == 0) j.int_array<uint8_t>(0, 255, data);
            else if (f == 1) j.int_array<uint64_t>(0, INT64_MAX, dims);
            else if (f == 2) { if (parse_params(j, p)) return DLLM_ERR_SERIALIZATION; }
            else j.skip_value();
        } while (j.ok && j.lit(","));
        j.expect('}');
    }
    j.ws();
    if (!j.ok || j.p != j.e) return fail(DLLM_ERR_SERIALIZATION, "json: malformed QuantizedTensor");
    for (bool v : seen)
        if (!v) return fail(DLLM_ERR_SERIALIZATION, "json: missing field of QuantizedTensor");
    *n = data.size();
    *ndim = dims.size();
    if (codes && codes_cap < data.size()) return fail(DLLM_ERR_INVALID_PARAMS, "codes buffer too small (see *n)");
    if (shape && shape_cap < dims.size()) return fail(DLLM_ERR_INVALID_PARAMS, "shape buffer too small (see *ndim)");
    if (codes && !data.empty()) std::memcpy(codes, data.data(), data.size());
    if (shape && !dims.empty()) std::memcpy(shape, dims.data(), dims.size() * 8);
    return DLLM_OK;
}

int dllm_compressed_vector_to_bincode(const char *id, size_t id_len, const uint8_t *data, size_t n, uint8_t bits,
                                      const uint64_t *shape, size_t ndim, float scale, float zero_point,
                                      uint8_t *out, size_t cap, size_t *len) {
    if ((!id && id_len) || (!data && n) || (!shape && ndim)) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    Writer w;
    w.bytes(reinterpret_cast<const uint8_t *>(id), id_len);
    w.bytes(data, n);
    w.u8(bits);
    w.usizes(shape, ndim);
    w.f32(scale);
    w.f32(zero_point);
    return emit(w.b, out, cap, len);
}

int dllm_compressed_vector_from_bincode(const uint8_t *buf, size_t len, int strict, char *id, size_t id_cap,
                                        size_t *id_len, uint8_t *data, size_t data_cap, size_t *n, uint8_t *bits,
                                        uint64_t *shape, size_t shape_cap, size_t *ndim, float *scale,
                                        float *zero_point) {
    if ((!buf && len) || !id_len || !n || !bits || !ndim || !scale || !zero_point)
        return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    Reader r{buf, len};
    auto vec = [&](void *dst, size_t cap, size_t *cnt) -> int {
        const uint64_t k = r.u64();
        if (!r.ok || k > len - r.i) return fail(DLLM_ERR_SERIALIZATION, "bincode: unexpected end of input");
        *cnt = k;
        if (dst && cap < k) return fail(DLLM_ERR_INVALID_PARAMS, "output buffer too small (see the count)");
        if (dst) r.take(dst, k);
        else r.i += k;
        return DLLM_OK;
    };
    if (const int rc = vec(id, id_cap, id_len)) return rc;
    if (id) {   // String: UTF-8 is checked by serde; an invalid sequence is a data error
        const unsigned char *u = reinterpret_cast<const unsigned char *>(id);
        for (size_t i = 0; i < *id_len;) {
            const size_t k = utf8_len(u + i, *id_len - i);
            if (!k) return fail(DLLM_ERR_SERIALIZATION, "bincode: invalid UTF-8 in String");
            i += k;
        }
    }
    if (const int rc = vec(data, data_cap, n)) return rc;
    *bits = r.u8();
    const uint64_t ns = r.u64();
    if (!r.ok || ns > (len - r.i) / 8) return fail(DLLM_ERR_SERIALIZATION, "bincode: unexpected end of input");
    *ndim = ns;
    if (shape && shape_cap < ns) return fail(DLLM_ERR_INVALID_PARAMS, "shape buffer too small (see *ndim)");
    for (uint64_t i = 0; i < ns; ++i) {
        const uint64_t v = r.u64();
        if (shape) shape[i] = v;
    }
    *scale = r.f32();
    *zero_point = r.f32();
    if (!r.ok) return fail(DLLM_ERR_SERIALIZATION, "bincode: unexpected end of input");
    return finish(r, strict, nullptr);
}

int dllm_compressed_vector_to_json(const char *id, size_t id_len, const uint8_t *data, size_t n, uint8_t bits,
                                   const uint64_t *shape, size_t ndim, float scale, float zero_point, char *out,
                                   size_t cap, size_t *len) {
    if ((!id && id_len) || (!data && n) || (!shape && ndim)) return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    const std::string s = "{\"id\":" + json_str(id, id_len) + ",\"data\":" + json_u8s(data, n) + ",\"bits\":" +
                          std::to_string(static_cast<unsigned>(bits)) + ",\"original_shape\":" + json_usizes(shape, ndim) +
                          ",\"quant_scale\":" + json_f32(scale) + ",\"quant_zero_point\":" + json_f32(zero_point) + "}";
    return emit(s, out, cap, len);
}

int dllm_compressed_vector_from_json(const char *s, size_t len, char *id, size_t id_cap, size_t *id_len,
                                     uint8_t *data, size_t data_cap, size_t *n, uint8_t *bits, uint64_t *shape,
                                     size_t shape_cap, size_t *ndim, float *scale, float *zero_point) {
    if ((!s && len) || !id_len || !n || !bits || !ndim || !scale || !zero_point)
        return fail(DLLM_ERR_INVALID_PARAMS, "null argument");
    JReader j{s, s + len};
    std::string ident;
    std::vector<uint8_t> codes;
    std::vector<uint64_t> dims;
    bool seen[6] = {false, false, false, false, false, false};
    j.expect('{');
    if (!j.lit("}")) {
        do {
            const std::string k = j.key();
            long long v;
            const int f = field_index(k, {"id", "data", "bits", "original_shape", "quant_scale", "quant_zero_point"});
            if (f >= 0 && seen[f]) return fail(DLLM_ERR_SERIALIZATION, "json: duplicate field of CompressedVector");
            if (f >= 0) seen[f] = true;
            if (f == 0) j.string(ident);
            else if (f == 1) j.int_array<uint8_t>(0, 255, codes);
            else if (f == 2) { if (j.integer(0, 255, v)) *bits = static_cast<uint8_t>(v); }
            else if (f == 3) j.int_array<uint64_t>(0, INT64_MAX, dims);
            else if (f == 4) *scale = j.f32_or_null();
            else if (f == 5) *zero_point = j.f32_or_null();
            else j.skip_value();
        } while (j.ok && j.lit(","));
        j.expect('}');
    }
    j.ws();
    if (!j.ok || j.p != j.e) return fail(DLLM_ERR_SERIALIZATION, "json: malformed CompressedVector");
    for (bool v : seen)
        if (!v) return fail(DLLM_ERR_SERIALIZATION, "json: missing field of CompressedVector");
    *id_len = ident.size();
    *n = codes.size();
    *ndim = dims.size();
    if ((id && id_cap < ident.size()) || (data && data_cap < codes.size()) || (shape && shape_cap < dims.size()))
        return fail(DLLM_ERR_INVALID_PARAMS, "output buffer too small (see the counts)");
    if (id && !ident.empty()) std::memcpy(id, ident.data(), ident.size());
    if (data && !codes.empty()) std::memcpy(data, codes.data(), codes.size());
    if (shape && !dims.empty()) std::memcpy(shape, dims.data(), dims.size() * 8);
    return DLLM_OK;
}

}  // extern "C"
