// wire.hpp -- JSON/base64 wire helpers shared by the native LSP client and the
// native miner (host-only C++, no HIP).
//
// Byte forms follow Go's encoding/json, which both reference apps use:
//   * lsp.Message (cmu440/lsp/message.go:20-27) marshals as
//     {"Type":..,"ConnID":..,"SeqNum":..,"Size":..,"Checksum":..,"Payload":<base64|null>}
//     ([]byte -> standard base64 with padding, nil -> null);
//   * bitcoin.Message (cmu440/bitcoin/message.go:18-23) marshals as
//     {"Type":..,"Data":"..","Lower":..,"Upper":..,"Hash":..,"Nonce":..}
//     with HTML-safe string escaping (<, >, & as <..; U+2028/9 escaped;
//     invalid UTF-8 bytes as �; other control bytes \u00XX except \n \r \t).
// Decoding is case-insensitive on keys and ignores unknown keys (Go).
#pragma once
#include <stdint.h>

#include <map>
#include <string>

namespace hm {
namespace wire {

std::string b64_encode(const std::string& bytes);
bool b64_decode(const std::string& text, std::string* out);

// Go encoding/json string literal (with quotes) of Go string bytes.
std::string json_string_go(const std::string& bytes);

struct JVal {
    enum Kind { NUL, NUM, STR, BOOL, OTHER } kind = NUL;
    std::string str;     // decoded UTF-8 bytes (STR) or the number's text (NUM)
    bool neg = false;
    uint64_t mag = 0;    // |value| when the number is an integer that fits
    bool int_ok = false; // integer literal (no fraction/exponent) within u64
    bool b = false;
};

// bitcoin.Message (cmu440/bitcoin/message.go:18-23) and its JSON forms.
struct BitcoinMsg {
    long long type = 0;  // Join 0, Request 1, Result 2 (message.go:9-13)
    std::string data;
    uint64_t lower = 0, upper = 0, hash = 0, nonce = 0;
};
std::string marshal_bitcoin(const BitcoinMsg& m);       // json.Marshal
// json.Unmarshal into a zero Message: a syntax error leaves the whole Message
// zero (Go validates before decoding), fields with type errors stay zero; the
// return value says whether the payload was valid JSON (the miner ignores it).
bool unmarshal_bitcoin(const std::string& payload, BitcoinMsg* m);

// Parse one flat JSON object; keys are lower-cased.  Returns false on syntax
// errors (values already parsed are kept, like Go's partial Unmarshal).
bool parse_object(const std::string& text, std::map<std::string, JVal>* out);

}  // namespace wire
}  // namespace hm
