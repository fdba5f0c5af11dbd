// Minimal JSON DOM used for the SceneData wire format.
//
// The reference passes scenes between its layers as plain JSON-able objects
// (`SceneData`, src/scenes/sceneData.ts:8-110; structured-cloned to workers in
// src/raytracer.ts:76-84). This is the C++ side of that wire format: numbers are
// IEEE doubles (JS `number`), objects keep insertion order, and serialisation
// prints doubles with 17 significant digits so a round trip is bit-exact.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace rtj {

struct Value;
using Member = std::pair<std::string, Value>;

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Value> arr;
    std::vector<Member> obj;

    Value() = default;
    static Value null() { return Value(); }
    static Value boolean(bool v) { Value x; x.kind = Bool; x.b = v; return x; }
    static Value number(double v) { Value x; x.kind = Number; x.num = v; return x; }
    static Value string(std::string v) { Value x; x.kind = String; x.str = std::move(v); return x; }
    static Value array() { Value x; x.kind = Array; return x; }
    static Value object() { Value x; x.kind = Object; return x; }

    bool is_null() const { return kind == Null; }
    bool is_number() const { return kind == Number; }
    bool is_string() const { return kind == String; }
    bool is_array() const { return kind == Array; }
    bool is_object() const { return kind == Object; }
    bool is_bool() const { return kind == Bool; }

    const Value* get(const char* key) const {
        if (kind != Object) return nullptr;
        for (const auto& m : obj)
            if (m.first == key) return &m.second;
        return nullptr;
    }
    Value& set(const std::string& key, Value v) {
        for (auto& m : obj)
            if (m.first == key) { m.second = std::move(v); return m.second; }
        obj.emplace_back(key, std::move(v));
        return obj.back().second;
    }
    Value& push(Value v) { arr.push_back(std::move(v)); return arr.back(); }
};

class ParseError : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

class Parser {
public:
    Parser(const char* s, size_t n) : p_(s), end_(s + n), begin_(s) {}
    Value parse_document() {
        Value v = parse_value();
        skip_ws();
        if (p_ != end_) fail("trailing characters");
        return v;
    }

private:
    const char* p_;
    const char* end_;
    const char* begin_;

    [[noreturn]] void fail(const char* what) {
        char buf[160];
        std::snprintf(buf, sizeof buf, "JSON parse error at offset %ld: %s",
                      (long)(p_ - begin_), what);
        throw ParseError(buf);
    }
    void skip_ws() {
        while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool lit(const char* s) {
        size_t n = std::strlen(s);
        if ((size_t)(end_ - p_) >= n && std::memcmp(p_, s, n) == 0) { p_ += n; return true; }
        return false;
    }
    Value parse_value() {
        skip_ws();
        if (p_ >= end_) fail("unexpected end");
        char c = *p_;
        if (c == '{') return parse_object();
        if (c == '[') return parse_array();
        if (c == '"') return Value::string(parse_string());
        if (lit("true")) return Value::boolean(true);
        if (lit("false")) return Value::boolean(false);
        if (lit("null")) return Value::null();
        // Non-standard tokens accepted so that JS-side Infinity/NaN survive a trip.
        if (lit("Infinity")) return Value::number(INFINITY);
        if (lit("-Infinity")) return Value::number(-INFINITY);
        if (lit("NaN")) return Value::number(NAN);
        return parse_number();
    }
    Value parse_number() {
        const char* start = p_;
        if (p_ < end_ && (*p_ == '-' || *p_ == '+')) ++p_;
        while (p_ < end_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' ||
                             *p_ == 'E' || *p_ == '-' || *p_ == '+'))
            ++p_;
        if (p_ == start) fail("invalid token");
        std::string tok(start, p_);
        char* e = nullptr;
        double v = std::strtod(tok.c_str(), &e);
        if (!e || *e != '\0') fail("invalid number");
        return Value::number(v);
    }
    static void put_utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) out.push_back((char)cp);
        else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
        else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    uint32_t hex4() {
        if (end_ - p_ < 4) fail("bad \\u escape");
        uint32_t v = 0;
        for (int i = 0; i < 4; ++i) {
            char c = *p_++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else fail("bad hex digit");
        }
        return v;
    }
    std::string parse_string() {
        ++p_;  // opening quote
        std::string out;
        while (true) {
            if (p_ >= end_) fail("unterminated string");
            char c = *p_++;
            if (c == '"') break;
            if (c != '\\') { out.push_back(c); continue; }
            if (p_ >= end_) fail("bad escape");
            char e = *p_++;
            switch (e) {
                case '"': out.push_back('"'); break;
                case '\\': out.push_back('\\'); break;
                case '/': out.push_back('/'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    uint32_t cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00 && end_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                        p_ += 2;
                        uint32_t lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    put_utf8(out, cp);
                    break;
                }
                default: fail("bad escape");
            }
        }
        return out;
    }
    Value parse_array() {
        ++p_;
        Value v = Value::array();
        skip_ws();
        if (p_ < end_ && *p_ == ']') { ++p_; return v; }
        while (true) {
            v.push(parse_value());
            skip_ws();
            if (p_ >= end_) fail("unterminated array");
            if (*p_ == ',') { ++p_; continue; }
            if (*p_ == ']') { ++p_; return v; }
            fail("expected , or ]");
        }
    }
    Value parse_object() {
        ++p_;
        Value v = Value::object();
        skip_ws();
        if (p_ < end_ && *p_ == '}') { ++p_; return v; }
        while (true) {
            skip_ws();
            if (p_ >= end_ || *p_ != '"') fail("expected key");
            std::string key = parse_string();
            skip_ws();
            if (p_ >= end_ || *p_ != ':') fail("expected :");
            ++p_;
            Value item = parse_value();
            v.set(key, std::move(item));
            skip_ws();
            if (p_ >= end_) fail("unterminated object");
            if (*p_ == ',') { ++p_; continue; }
            if (*p_ == '}') { ++p_; return v; }
            fail("expected , or }");
        }
    }
};

inline Value parse(const std::string& s) { return Parser(s.data(), s.size()).parse_document(); }
inline Value parse(const char* s, size_t n) { return Parser(s, n).parse_document(); }

inline void dump_string(std::string& out, const std::string& s) {
    out.push_back('"');
    for (unsigned char c : s) {
        switch (c) {
            case '"': out += "\\\""; break;
            case '\\': out += "\\\\"; break;
            case '\n': out += "\\n"; break;
            case '\r': out += "\\r"; break;
            case '\t': out += "\\t"; break;
            default:
                if (c < 0x20) { char b[8]; std::snprintf(b, sizeof b, "\\u%04x", c); out += b; }
                else out.push_back((char)c);
        }
    }
    out.push_back('"');
}

inline void dump_number(std::string& out, double v) {
    if (std::isnan(v)) { out += "NaN"; return; }
    if (std::isinf(v)) { out += v > 0 ? "Infinity" : "-Infinity"; return; }
    if (v == std::floor(v) && std::fabs(v) < 1e15) {
        char b[32];
        std::snprintf(b, sizeof b, "%.0f", v);
        if (v == 0 && std::signbit(v)) { out += "-0"; return; }
        out += b;
        return;
    }
    char b[40];
    std::snprintf(b, sizeof b, "%.17g", v);
    out += b;
}

inline void dump(std::string& out, const Value& v) {
    switch (v.kind) {
        case Value::Null: out += "null"; break;
        case Value::Bool: out += v.b ? "true" : "false"; break;
        case Value::Number: dump_number(out, v.num); break;
        case Value::String: dump_string(out, v.str); break;
        case Value::Array:
            out.push_back('[');
            for (size_t i = 0; i < v.arr.size(); ++i) {
                if (i) out.push_back(',');
                dump(out, v.arr[i]);
            }
            out.push_back(']');
            break;
        case Value::Object:
            out.push_back('{');
            for (size_t i = 0; i < v.obj.size(); ++i) {
                if (i) out.push_back(',');
                dump_string(out, v.obj[i].first);
                out.push_back(':');
                dump(out, v.obj[i].second);
            }
            out.push_back('}');
            break;
    }
}

inline std::string dump(const Value& v) {
    std::string s;
    dump(s, v);
    return s;
}

inline Value vec3(double x, double y, double z) {
    Value a = Value::array();
    a.push(Value::number(x));
    a.push(Value::number(y));
    a.push(Value::number(z));
    return a;
}

}  // namespace rtj
