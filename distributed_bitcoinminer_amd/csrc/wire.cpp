// wire.cpp -- see wire.hpp.
#include "wire.hpp"

#include <stdio.h>
#include <string.h>

namespace hm {
namespace wire {

static const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string b64_encode(const std::string& in) {
    std::string out;
    out.reserve((in.size() + 2) / 3 * 4);
    size_t i = 0;
    for (; i + 3 <= in.size(); i += 3) {
        const uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
        out += kB64[v >> 18]; out += kB64[(v >> 12) & 63];
        out += kB64[(v >> 6) & 63]; out += kB64[v & 63];
    }
    const size_t rem = in.size() - i;
    if (rem == 1) {
        const uint32_t v = (uint8_t)in[i] << 16;
        out += kB64[v >> 18]; out += kB64[(v >> 12) & 63]; out += "==";
    } else if (rem == 2) {
        const uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
        out += kB64[v >> 18]; out += kB64[(v >> 12) & 63]; out += kB64[(v >> 6) & 63]; out += '=';
    }
    return out;
}

static int b64_val(char c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
}

bool b64_decode(const std::string& t, std::string* out) {
    out->clear();
    if (t.size() % 4) return false;
    for (size_t i = 0; i < t.size(); i += 4) {
        int v[4];
        int pad = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = t[i + k];
            if (c == '=' && i + 4 == t.size() && k >= 2) { v[k] = 0; ++pad; continue; }
            if (pad) return false;
            v[k] = b64_val(c);
            if (v[k] < 0) return false;
        }
        const uint32_t x = (v[0] << 18) | (v[1] << 12) | (v[2] << 6) | v[3];
        out->push_back((char)(x >> 16));
        if (pad < 2) out->push_back((char)((x >> 8) & 255));
        if (pad < 1) out->push_back((char)(x & 255));
    }
    return true;
}

// utf8.DecodeRune: rune and size, or -1 with size 1 for an invalid byte.
static int decode_rune(const std::string& s, size_t i, size_t* size) {
    const uint8_t c = (uint8_t)s[i];
    int n = 0;
    uint32_t r = 0, min = 0;
    if (c >= 0xC2 && c <= 0xDF) { n = 2; r = c & 0x1F; min = 0x80; }
    else if (c >= 0xE0 && c <= 0xEF) { n = 3; r = c & 0x0F; min = 0x800; }
    else if (c >= 0xF0 && c <= 0xF4) { n = 4; r = c & 0x07; min = 0x10000; }
    else { *size = 1; return -1; }
    if (i + n > s.size()) { *size = 1; return -1; }
    for (int k = 1; k < n; ++k) {
        const uint8_t cc = (uint8_t)s[i + k];
        if ((cc & 0xC0) != 0x80) { *size = 1; return -1; }
        r = (r << 6) | (cc & 0x3F);
    }
    if (r < min || r > 0x10FFFF || (r >= 0xD800 && r <= 0xDFFF)) { *size = 1; return -1; }
    *size = (size_t)n;
    return (int)r;
}

std::string json_string_go(const std::string& b) {
    static const char hex[] = "0123456789abcdef";
    std::string out = "\"";
    for (size_t i = 0; i < b.size();) {
        const uint8_t c = (uint8_t)b[i];
        if (c < 0x80) {
            switch (c) {
                case '"': out += "\\\""; break;
                case '\\': out += "\\\\"; break;
                case '\n': out += "\\n"; break;
                case '\r': out += "\\r"; break;
                case '\t': out += "\\t"; break;
                default:
                    if (c < 0x20 || c == '<' || c == '>' || c == '&') {
                        out += "\\u00";
                        out += hex[c >> 4];
                        out += hex[c & 15];
                    } else {
                        out += (char)c;
                    }
            }
            ++i;
            continue;
        }
        size_t n = 1;
        const int r = decode_rune(b, i, &n);
        if (r < 0) out += "\\ufffd";
        else if (r == 0x2028) out += "\\u2028";
        else if (r == 0x2029) out += "\\u2029";
        else out.append(b, i, n);
        i += n;
    }
    out += '"';
    return out;
}

// ---------------------------------------------------------------------------
// Minimal JSON object parser (flat objects of scalars; nested values skipped)
// ---------------------------------------------------------------------------
namespace {

struct P {
    const std::string& s;
    size_t i = 0;
    explicit P(const std::string& x) : s(x) {}
    void ws() { while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i; }
    bool eat(char c) { ws(); if (i < s.size() && s[i] == c) { ++i; return true; } return false; }
};

void put_utf8(std::string* o, uint32_t r) {
    if (r < 0x80) o->push_back((char)r);
    else if (r < 0x800) { o->push_back((char)(0xC0 | (r >> 6))); o->push_back((char)(0x80 | (r & 63))); }
    else if (r < 0x10000) {
        o->push_back((char)(0xE0 | (r >> 12))); o->push_back((char)(0x80 | ((r >> 6) & 63)));
        o->push_back((char)(0x80 | (r & 63)));
    } else {
        o->push_back((char)(0xF0 | (r >> 18))); o->push_back((char)(0x80 | ((r >> 12) & 63)));
        o->push_back((char)(0x80 | ((r >> 6) & 63))); o->push_back((char)(0x80 | (r & 63)));
    }
}

bool hex4(P& p, uint32_t* v) {
    if (p.i + 4 > p.s.size()) return false;
    uint32_t x = 0;
    for (int k = 0; k < 4; ++k) {
        const char c = p.s[p.i + k];
        x <<= 4;
        if (c >= '0' && c <= '9') x |= c - '0';
        else if (c >= 'a' && c <= 'f') x |= c - 'a' + 10;
        else if (c >= 'A' && c <= 'F') x |= c - 'A' + 10;
        else return false;
    }
    p.i += 4;
    *v = x;
    return true;
}

// Go's unquote: escapes decoded, lone surrogates and invalid UTF-8 -> U+FFFD.
bool parse_string(P& p, std::string* out) {
    out->clear();
    if (!p.eat('"')) return false;
    while (p.i < p.s.size()) {
        const uint8_t c = (uint8_t)p.s[p.i];
        if (c == '"') { ++p.i; return true; }
        if (c < 0x20) return false;
        if (c == '\\') {
            if (++p.i >= p.s.size()) return false;
            const char e = p.s[p.i++];
            switch (e) {
                case '"': out->push_back('"'); break;
                case '\\': out->push_back('\\'); break;
                case '/': out->push_back('/'); break;
                case 'b': out->push_back('\b'); break;
                case 'f': out->push_back('\f'); break;
                case 'n': out->push_back('\n'); break;
                case 'r': out->push_back('\r'); break;
                case 't': out->push_back('\t'); break;
                case 'u': {
                    uint32_t r;
                    if (!hex4(p, &r)) return false;
                    if (r >= 0xD800 && r < 0xDC00 && p.i + 6 <= p.s.size() && p.s[p.i] == '\\' &&
                        p.s[p.i + 1] == 'u') {
                        const size_t save = p.i;
                        p.i += 2;
                        uint32_t r2;
                        if (hex4(p, &r2) && r2 >= 0xDC00 && r2 < 0xE000) {
                            r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
                        } else {
                            p.i = save;
                            r = 0xFFFD;
                        }
                    } else if (r >= 0xD800 && r < 0xE000) {
                        r = 0xFFFD;
                    }
                    put_utf8(out, r);
                    break;
                }
                default: return false;
            }
            continue;
        }
        if (c < 0x80) { out->push_back((char)c); ++p.i; continue; }
        size_t n = 1;
        const int r = decode_rune(p.s, p.i, &n);
        if (r < 0) { put_utf8(out, 0xFFFD); p.i += 1; }
        else { out->append(p.s, p.i, n); p.i += n; }
    }
    return false;
}

bool skip_value(P& p, int depth);

bool parse_value(P& p, JVal* v, int depth) {
    p.ws();
    if (p.i >= p.s.size()) return false;
    const char c = p.s[p.i];
    if (c == '"') { v->kind = JVal::STR; return parse_string(p, &v->str); }
    if (c == 'n' && p.s.compare(p.i, 4, "null") == 0) { p.i += 4; v->kind = JVal::NUL; return true; }
    if (c == 't' && p.s.compare(p.i, 4, "true") == 0) { p.i += 4; v->kind = JVal::BOOL; v->b = true; return true; }
    if (c == 'f' && p.s.compare(p.i, 5, "false") == 0) { p.i += 5; v->kind = JVal::BOOL; return true; }
    if (c == '-' || (c >= '0' && c <= '9')) {
        const size_t st = p.i;
        v->kind = JVal::NUM;
        v->neg = (c == '-');
        if (v->neg) ++p.i;
        uint64_t mag = 0;
        bool ok = true, digits = false;
        while (p.i < p.s.size() && p.s[p.i] >= '0' && p.s[p.i] <= '9') {
            const uint64_t d = (uint64_t)(p.s[p.i] - '0');
            if (mag > (~0ull - d) / 10) ok = false;
            mag = mag * 10 + d;
            digits = true;
            ++p.i;
        }
        if (!digits) return false;
        bool frac = false;
        if (p.i < p.s.size() && p.s[p.i] == '.') {
            frac = true;
            ++p.i;
            while (p.i < p.s.size() && p.s[p.i] >= '0' && p.s[p.i] <= '9') ++p.i;
        }
        if (p.i < p.s.size() && (p.s[p.i] == 'e' || p.s[p.i] == 'E')) {
            frac = true;
            ++p.i;
            if (p.i < p.s.size() && (p.s[p.i] == '+' || p.s[p.i] == '-')) ++p.i;
            while (p.i < p.s.size() && p.s[p.i] >= '0' && p.s[p.i] <= '9') ++p.i;
        }
        v->str = p.s.substr(st, p.i - st);
        v->mag = mag;
        v->int_ok = ok && !frac;
        return true;
    }
    v->kind = JVal::OTHER;
    return skip_value(p, depth);
}

bool skip_value(P& p, int depth) {
    if (depth > 64) return false;
    p.ws();
    if (p.i >= p.s.size()) return false;
    const char c = p.s[p.i];
    if (c == '{' || c == '[') {
        const char close = c == '{' ? '}' : ']';
        ++p.i;
        if (p.eat(close)) return true;
        for (;;) {
            if (c == '{') {
                std::string k;
                if (!parse_string(p, &k) || !p.eat(':')) return false;
            }
            if (!skip_value(p, depth + 1)) return false;
            if (p.eat(close)) return true;
            if (!p.eat(',')) return false;
        }
    }
    JVal tmp;
    return parse_value(p, &tmp, depth + 1);
}

}  // namespace

bool parse_object(const std::string& text, std::map<std::string, JVal>* out) {
    P p(text);
    if (!p.eat('{')) return false;
    if (p.eat('}')) return true;
    for (;;) {
        std::string key;
        if (!parse_string(p, &key) || !p.eat(':')) return false;
        JVal v;
        if (!parse_value(p, &v, 0)) return false;
        for (auto& ch : key) ch = (char)((ch >= 'A' && ch <= 'Z') ? ch - 'A' + 'a' : ch);
        (*out)[key] = v;
        if (p.eat('}')) break;
        if (!p.eat(',')) return false;
    }
    p.ws();
    return p.i == text.size();
}

std::string marshal_bitcoin(const BitcoinMsg& m) {
    char nums[200];
    std::string out = "{\"Type\":" + std::to_string(m.type) + ",\"Data\":" + json_string_go(m.data);
    snprintf(nums, sizeof nums, ",\"Lower\":%llu,\"Upper\":%llu,\"Hash\":%llu,\"Nonce\":%llu}",
             (unsigned long long)m.lower, (unsigned long long)m.upper,
             (unsigned long long)m.hash, (unsigned long long)m.nonce);
    return out + nums;
}

bool unmarshal_bitcoin(const std::string& payload, BitcoinMsg* m) {
    *m = BitcoinMsg();
    std::map<std::string, JVal> o;
    // Go's Unmarshal validates the whole input first: a syntax error decodes
    // nothing; type errors on single fields leave just those fields zero.
    const bool ok = parse_object(payload, &o);
    if (!ok) return false;
    auto u64 = [&](const char* k, uint64_t* dst) {
        auto it = o.find(k);
        if (it != o.end() && it->second.kind == JVal::NUM && it->second.int_ok && !it->second.neg)
            *dst = it->second.mag;
    };
    auto it = o.find("type");
    if (it != o.end() && it->second.kind == JVal::NUM && it->second.int_ok &&
        it->second.mag <= 0x7fffffffffffffffull)
        m->type = it->second.neg ? -(long long)it->second.mag : (long long)it->second.mag;
    it = o.find("data");
    if (it != o.end() && it->second.kind == JVal::STR) m->data = it->second.str;
    u64("lower", &m->lower);
    u64("upper", &m->upper);
    u64("hash", &m->hash);
    u64("nonce", &m->nonce);
    return true;
}

}  // namespace wire
}  // namespace hm
