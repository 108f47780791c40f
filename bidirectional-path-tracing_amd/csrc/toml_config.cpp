// Scene configuration from the reference's TOML files: loadTOML (reference
// src/main.cpp:22-116) over cpptoml (externals/cpptoml.h) and the objfile
// resolution of Scene::load (src/core/renderer.cpp:235-241).
//
// The parser covers the TOML the reference reads: [tables], bare / quoted
// keys, basic and literal strings, integers, floats, booleans and (possibly
// multi-line) arrays; dates, inline tables and multi-line strings are rejected
// with an error. Typed reads follow cpptoml's get_as / get_array_of:
//   get_as<double>   accepts a float, or an integer converted to double
//                    (cpptoml.h:694-713); anything else -> the default;
//   get_as<int>      accepts an integer only (range-checked, cpptoml.h:1221-1238);
//                    a float -> the default;
//   get_array_of<double>  every element must convert, else the default
//                    (cpptoml.h:1481-1500); arrays must be homogeneous (:3048).
// Floats are parsed as double by strtod (cpptoml parse_float uses std::stod,
// :2810-2820) and then narrowed to float where the reference's Config field is
// float — the same double rounding as the reference.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "bdpt_amd.h"
#include "scene.hpp"

namespace bdpt {
namespace {

struct Value {
    enum Kind { STRING, INT, FLOAT, BOOL, ARRAY } kind = STRING;
    std::string s;
    int64_t i = 0;
    double f = 0.0;
    bool b = false;
    std::vector<Value> arr;
    Kind elem = STRING;  // arrays: element type fixed by the first element (cpptoml)
};

typedef std::map<std::string, Value> Table;

class Parser {
   public:
    Parser(const std::string& text, std::map<std::string, Table>& out) : t_(text), out_(out) {}

    bool run(std::string& err) {
        std::string table;  // root table = ""
        out_[table];
        while (true) {
            skip_ws_nl_comments();
            if (p_ >= t_.size()) return true;
            if (t_[p_] == '[') {
                if (p_ + 1 < t_.size() && t_[p_ + 1] == '[') return fail(err, "arrays of tables are not supported");
                p_++;
                skip_ws();
                std::string name;
                if (!read_key(name, err)) return false;
                while (skip_ws(), p_ < t_.size() && t_[p_] == '.') {
                    p_++;
                    skip_ws();
                    std::string part;
                    if (!read_key(part, err)) return false;
                    name += "." + part;
                }
                if (p_ >= t_.size() || t_[p_] != ']') return fail(err, "expected ']' after table name");
                p_++;
                if (out_.count(name) && defined_.count(name)) return fail(err, "table [" + name + "] defined twice");
                defined_.insert({name, true});
                table = name;
                out_[table];
                if (!end_of_line(err)) return false;
                continue;
            }
            std::string key;
            if (!read_key(key, err)) return false;
            skip_ws();
            if (p_ >= t_.size() || t_[p_] != '=') return fail(err, "expected '=' after key '" + key + "'");
            p_++;
            skip_ws();
            Value v;
            if (!read_value(v, err)) return false;
            Table& tb = out_[table];
            if (tb.count(key)) return fail(err, "key '" + key + "' already present");
            tb[key] = v;
            if (!end_of_line(err)) return false;
        }
    }

   private:
    const std::string& t_;
    std::map<std::string, Table>& out_;
    std::map<std::string, bool> defined_;
    size_t p_ = 0;
    int line_ = 1;

    bool fail(std::string& err, const std::string& msg) {
        err = msg + " (line " + std::to_string(line_) + ")";
        return false;
    }
    void skip_ws() {
        while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\t')) p_++;
    }
    void skip_comment() {
        if (p_ < t_.size() && t_[p_] == '#')
            while (p_ < t_.size() && t_[p_] != '\n') p_++;
    }
    void skip_ws_nl_comments() {
        for (;;) {
            skip_ws();
            skip_comment();
            if (p_ < t_.size() && (t_[p_] == '\n' || t_[p_] == '\r')) {
                if (t_[p_] == '\n') line_++;
                p_++;
                continue;
            }
            return;
        }
    }
    bool end_of_line(std::string& err) {
        skip_ws();
        skip_comment();
        if (p_ < t_.size() && t_[p_] == '\r') p_++;
        if (p_ < t_.size() && t_[p_] != '\n') return fail(err, "unexpected characters after value");
        return true;
    }
    bool read_key(std::string& key, std::string& err) {
        if (p_ < t_.size() && (t_[p_] == '"' || t_[p_] == '\'')) {
            Value v;
            if (!read_string(v, err)) return false;
            key = v.s;
            return true;
        }
        const size_t b = p_;
        while (p_ < t_.size() && (std::isalnum(static_cast<unsigned char>(t_[p_])) || t_[p_] == '_' || t_[p_] == '-'))
            p_++;
        if (p_ == b) return fail(err, "expected a key");
        key = t_.substr(b, p_ - b);
        return true;
    }
    static void put_utf8(std::string& s, uint32_t c) {
        if (c < 0x80) s += static_cast<char>(c);
        else if (c < 0x800) s += static_cast<char>(0xc0 | (c >> 6)), s += static_cast<char>(0x80 | (c & 0x3f));
        else if (c < 0x10000)
            s += static_cast<char>(0xe0 | (c >> 12)), s += static_cast<char>(0x80 | ((c >> 6) & 0x3f)),
                s += static_cast<char>(0x80 | (c & 0x3f));
        else
            s += static_cast<char>(0xf0 | (c >> 18)), s += static_cast<char>(0x80 | ((c >> 12) & 0x3f)),
                s += static_cast<char>(0x80 | ((c >> 6) & 0x3f)), s += static_cast<char>(0x80 | (c & 0x3f));
    }
    bool read_string(Value& v, std::string& err) {
        const char q = t_[p_];
        if (t_.compare(p_, 3, std::string(3, q)) == 0) return fail(err, "multi-line strings are not supported");
        p_++;
        v.kind = Value::STRING;
        v.s.clear();
        while (p_ < t_.size() && t_[p_] != q) {
            char c = t_[p_++];
            if (c == '\n') return fail(err, "unterminated string");
            if (q == '"' && c == '\\') {
                if (p_ >= t_.size()) return fail(err, "unterminated string");
                const char e = t_[p_++];
                switch (e) {
                    case 'b': v.s += '\b'; break;
                    case 't': v.s += '\t'; break;
                    case 'n': v.s += '\n'; break;
                    case 'f': v.s += '\f'; break;
                    case 'r': v.s += '\r'; break;
                    case '"': v.s += '"'; break;
                    case '\\': v.s += '\\'; break;
                    case 'u':
                    case 'U': {
                        const int n = e == 'u' ? 4 : 8;
                        if (p_ + n > t_.size()) return fail(err, "bad unicode escape");
                        const std::string hex = t_.substr(p_, n);
                        for (char h : hex)
                            if (!std::isxdigit(static_cast<unsigned char>(h))) return fail(err, "bad unicode escape");
                        put_utf8(v.s, static_cast<uint32_t>(std::strtoul(hex.c_str(), nullptr, 16)));
                        p_ += n;
                        break;
                    }
                    default: return fail(err, std::string("invalid escape sequence \\") + e);
                }
                continue;
            }
            v.s += c;
        }
        if (p_ >= t_.size()) return fail(err, "unterminated string");
        p_++;
        return true;
    }
    bool read_number(Value& v, std::string& err) {
        const size_t b = p_;
        while (p_ < t_.size() && (std::isalnum(static_cast<unsigned char>(t_[p_])) || t_[p_] == '+' ||
                                  t_[p_] == '-' || t_[p_] == '.' || t_[p_] == '_' || t_[p_] == ':'))
            p_++;
        std::string tok = t_.substr(b, p_ - b);
        if (tok.empty()) return fail(err, "expected a value");
        if (tok.find(':') != std::string::npos || (tok.size() >= 10 && tok[4] == '-' && tok[7] == '-'))
            return fail(err, "dates are not supported");
        std::string clean;
        for (size_t k = 0; k < tok.size(); k++) {
            if (tok[k] == '_') {
                const bool ok = k > 0 && k + 1 < tok.size() && std::isalnum(static_cast<unsigned char>(tok[k - 1])) &&
                                std::isalnum(static_cast<unsigned char>(tok[k + 1]));
                if (!ok) return fail(err, "malformed number '" + tok + "'");
                continue;
            }
            clean += tok[k];
        }
        const std::string body = (clean[0] == '+' || clean[0] == '-') ? clean.substr(1) : clean;
        if (body == "inf" || body == "nan") {
            v.kind = Value::FLOAT;
            v.f = body == "inf" ? HUGE_VAL : NAN;
            if (clean[0] == '-') v.f = -v.f;
            return true;
        }
        const bool is_float = body.find_first_of(".eE") != std::string::npos && body.compare(0, 2, "0x") != 0;
        char* end = nullptr;
        errno = 0;
        if (is_float) {
            if (body.empty() || !std::isdigit(static_cast<unsigned char>(body[0])) || body.back() == '.')
                return fail(err, "malformed float '" + tok + "'");
            const size_t dot = body.find('.');
            if (dot != std::string::npos && (dot + 1 >= body.size() || !std::isdigit(static_cast<unsigned char>(body[dot + 1]))))
                return fail(err, "malformed float '" + tok + "'");
            v.kind = Value::FLOAT;
            v.f = std::strtod(clean.c_str(), &end);
            if (*end) return fail(err, "malformed float '" + tok + "'");
            return true;
        }
        int base = 10;
        std::string digits = clean;
        if (body.size() > 2 && body[0] == '0' && (body[1] == 'x' || body[1] == 'o' || body[1] == 'b')) {
            if (clean[0] == '+' || clean[0] == '-') return fail(err, "signed non-decimal integer '" + tok + "'");
            base = body[1] == 'x' ? 16 : (body[1] == 'o' ? 8 : 2);
            digits = body.substr(2);
        } else if (body.size() > 1 && body[0] == '0') {
            return fail(err, "leading zero in integer '" + tok + "'");
        }
        for (char c : (base == 10 ? body : digits)) {
            const bool ok = base == 16 ? std::isxdigit(static_cast<unsigned char>(c)) != 0
                                       : (c >= '0' && c < static_cast<char>('0' + (base > 10 ? 10 : base)));
            if (!ok) return fail(err, "malformed integer '" + tok + "'");
        }
        v.kind = Value::INT;
        v.i = static_cast<int64_t>(std::strtoll(digits.c_str(), &end, base));
        if (errno == ERANGE || *end) return fail(err, "integer out of range '" + tok + "'");
        return true;
    }
    // determine_value_type / determine_number_type (cpptoml.h:2312-2381) of the
    // value starting at the cursor.
    Value::Kind first_element_kind() const {
        size_t q = p_;
        if (q >= t_.size()) return Value::STRING;
        const char c = t_[q];
        if (c == '"' || c == '\'') return Value::STRING;
        if (c == 't' || c == 'f') return Value::BOOL;
        if (c == '[') return Value::ARRAY;
        if (c == '+' || c == '-') q++;
        if (q < t_.size() && (t_[q] == 'i' || t_[q] == 'n')) return Value::FLOAT;
        while (q < t_.size() && std::isdigit(static_cast<unsigned char>(t_[q]))) q++;
        return (q < t_.size() && t_[q] == '.') ? Value::FLOAT : Value::INT;
    }

    bool read_value(Value& v, std::string& err) {
        if (p_ >= t_.size()) return fail(err, "expected a value");
        const char c = t_[p_];
        if (c == '"' || c == '\'') return read_string(v, err);
        if (c == '{') return fail(err, "inline tables are not supported");
        if (c == '[') {
            p_++;
            v.kind = Value::ARRAY;
            for (;;) {
                skip_ws_nl_comments();
                if (p_ < t_.size() && t_[p_] == ']') {
                    p_++;
                    return true;
                }
                // cpptoml (:2985-3051) fixes the element type from the FIRST element's
                // text (a number is FLOAT only if its digits are followed by '.', or it
                // is inf / nan, :2355-2381), then requires as<T>() of every element:
                // a FLOAT array also takes integers, an INT array takes no floats.
                if (v.arr.empty()) v.elem = first_element_kind();
                Value e;
                if (!read_value(e, err)) return false;
                const bool ok = e.kind == v.elem || (v.elem == Value::FLOAT && e.kind == Value::INT);
                if (!ok) return fail(err, "Arrays must be homogeneous");
                v.arr.push_back(e);
                skip_ws_nl_comments();
                if (p_ < t_.size() && t_[p_] == ',') {
                    p_++;
                    continue;
                }
                if (p_ < t_.size() && t_[p_] == ']') {
                    p_++;
                    return true;
                }
                return fail(err, "expected ',' or ']' in array");
            }
        }
        if (t_.compare(p_, 4, "true") == 0 && !std::isalnum(static_cast<unsigned char>(p_ + 4 < t_.size() ? t_[p_ + 4] : ' '))) {
            p_ += 4;
            v.kind = Value::BOOL;
            v.b = true;
            return true;
        }
        if (t_.compare(p_, 5, "false") == 0 && !std::isalnum(static_cast<unsigned char>(p_ + 5 < t_.size() ? t_[p_ + 5] : ' '))) {
            p_ += 5;
            v.kind = Value::BOOL;
            v.b = false;
            return true;
        }
        return read_number(v, err);
    }
};

// cpptoml typed reads (see the header comment).
const Value* find(const Table* t, const char* key) {
    if (!t) return nullptr;
    auto it = t->find(key);
    return it == t->end() ? nullptr : &it->second;
}
double get_double(const Table* t, const char* key, double dflt) {
    const Value* v = find(t, key);
    if (v && v->kind == Value::FLOAT) return v->f;
    if (v && v->kind == Value::INT) return static_cast<double>(v->i);
    return dflt;
}
bool get_int(const Table* t, const char* key, int dflt, int& out, std::string& err) {
    const Value* v = find(t, key);
    out = dflt;
    if (!v || v->kind != Value::INT) return true;
    if (v->i < INT32_MIN || v->i > INT32_MAX) {
        err = std::string("T cannot represent the value requested in get (") + key + ")";
        return false;
    }
    out = static_cast<int>(v->i);
    return true;
}
bool get_bool(const Table* t, const char* key, bool dflt) {
    const Value* v = find(t, key);
    return (v && v->kind == Value::BOOL) ? v->b : dflt;
}
std::vector<double> get_array_double(const Table* t, const char* key, const std::vector<double>& dflt) {
    const Value* v = find(t, key);
    if (!v || v->kind != Value::ARRAY) return dflt;
    std::vector<double> r;
    for (const Value& e : v->arr) {
        if (e.kind == Value::FLOAT) r.push_back(e.f);
        else if (e.kind == Value::INT) r.push_back(static_cast<double>(e.i));
        else return dflt;
    }
    return r;
}

void copy_str(char* dst, size_t cap, const std::string& s) {
    std::strncpy(dst, s.c_str(), cap - 1);
    dst[cap - 1] = '\0';
}

}  // namespace

bool load_toml_config(const std::string& path, bdpt_config& cfg, std::string& err) {
    std::ifstream in(path, std::ios::binary);
    if (!in) {
        err = "cannot open " + path;
        return false;
    }
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string text = ss.str();
    std::map<std::string, Table> tables;
    Parser P(text, tables);
    if (!P.run(err)) {
        err = path + ": " + err;
        return false;
    }
    auto table = [&](const char* n) -> const Table* {
        auto it = tables.find(n);
        return it == tables.end() ? nullptr : &it->second;
    };
    std::memset(&cfg, 0, sizeof(cfg));
    copy_str(cfg.toml_file, sizeof(cfg.toml_file), path);
    // [input] objfile (main.cpp:26-27): required — the reference dereferences the option.
    const Table* input = table("input");
    const Value* obj = find(input, "objfile");
    if (!input || !obj || obj->kind != Value::STRING) {
        err = path + ": [input] objfile missing";
        return false;
    }
    copy_str(cfg.obj_file_raw, sizeof(cfg.obj_file_raw), obj->s);
    // Scene::load (renderer.cpp:236-241): a relative objfile resolves against the TOML's directory.
    std::string resolved = obj->s;
    if (resolved.empty() || resolved[0] != '/') {
        const size_t slash = path.find_last_of('/');
        resolved = (slash == std::string::npos ? std::string() : path.substr(0, slash + 1)) + resolved;
    }
    copy_str(cfg.obj_file, sizeof(cfg.obj_file), resolved);
    // The reference dereferences these tables unconditionally (main.cpp:30, :40, :45).
    const Table* camera = table("camera");
    const Table* film = table("film");
    const Table* renderer = table("renderer");
    if (!camera || !film || !renderer) {
        err = path + ": [camera], [film] and [renderer] tables are required";
        return false;
    }
    // [camera] (main.cpp:30-37)
    cfg.camera.fov = static_cast<float>(get_double(camera, "fov", 30.));
    const char* names[3] = {"eye", "at", "up"};
    const std::vector<double> dflt[3] = {{1., 1., 0.}, {0., 0., 0.}, {0., 1., 0.}};
    float* dst[3] = {cfg.camera.eye, cfg.camera.at, cfg.camera.up};
    for (int k = 0; k < 3; k++) {
        const std::vector<double> a = get_array_double(camera, names[k], dflt[k]);
        if (a.size() < 3) {
            err = path + ": [camera] " + names[k] + " needs 3 numbers";
            return false;
        }
        for (int c = 0; c < 3; c++) dst[k][c] = static_cast<float>(a[c]);
    }
    // [film] (main.cpp:40-42)
    if (!get_int(film, "width", 768, cfg.width, err) || !get_int(film, "height", 576, cfg.height, err)) return false;
    // [renderer] (main.cpp:45-113)
    cfg.realtime = get_bool(renderer, "realtime", false) ? 1 : 0;
    const Value* type = find(renderer, "type");
    copy_str(cfg.integrator, sizeof(cfg.integrator), (type && type->kind == Value::STRING) ? type->s : "normal");
    cfg.rr_depth = 5;
    cfg.rr_prob = 0.f;
    cfg.spp = 1;
    cfg.path = bdpt_path_params{1, -1, 5, 0.95f, 1, 0};
    cfg.direct = bdpt_direct_params{0, 1, 1};
    copy_str(cfg.sampling_strategy, sizeof(cfg.sampling_strategy), "emitter");
    if (!cfg.realtime) {
        const std::string t = cfg.integrator;
        static const char* known[] = {"normal", "simple", "ao", "ro", "direct", "path", "bdpt"};
        bool ok = false;
        for (const char* k : known) ok = ok || t == k;
        if (!ok) {
            err = "Invalid integrator type";  // main.cpp:109
            return false;
        }
        if (t == "bdpt") {  // main.cpp:103-107
            if (!get_int(renderer, "rrDepth", 5, cfg.rr_depth, err)) return false;
            cfg.rr_prob = static_cast<float>(get_double(renderer, "rrProb", 0.f));
        } else if (t == "path") {  // main.cpp:96-101
            if (!get_int(renderer, "rrDepth", 5, cfg.rr_depth, err)) return false;
            cfg.rr_prob = static_cast<float>(get_double(renderer, "rrProb", 0.95f));
            cfg.path.is_explicit = get_bool(renderer, "isExplicit", true) ? 1 : 0;
            if (!get_int(renderer, "maxDepth", -1, cfg.path.max_depth, err)) return false;
            // get_as<size_t>: a negative integer throws (cpptoml.h:1245-1262)
            if (!get_int(renderer, "emitterSamples", 1, cfg.path.emitter_samples, err) ||
                !get_int(renderer, "bsdfSamples", 0, cfg.path.bsdf_samples, err))
                return false;
            if (cfg.path.emitter_samples < 0 || cfg.path.bsdf_samples < 0) {
                err = "T cannot store negative value in get";
                return false;
            }
            cfg.path.rr_depth = cfg.rr_depth;
            cfg.path.rr_prob = cfg.rr_prob;
        } else if (t == "direct") {  // main.cpp:88-92
            if (!get_int(renderer, "emitterSamples", 1, cfg.direct.emitter_samples, err) ||
                !get_int(renderer, "bsdfSamples", 1, cfg.direct.bsdf_samples, err))
                return false;
            if (cfg.direct.emitter_samples < 0 || cfg.direct.bsdf_samples < 0) {
                err = "T cannot store negative value in get";
                return false;
            }
            const Value* ss = find(renderer, "samplingStrategy");
            copy_str(cfg.sampling_strategy, sizeof(cfg.sampling_strategy),
                     (ss && ss->kind == Value::STRING) ? ss->s : "emitter");
            cfg.direct.sampling_strategy = bdpt_direct_strategy(cfg.sampling_strategy);
        }
        if (!get_int(renderer, "spp", 1, cfg.spp, err)) return false;  // main.cpp:112
    }
    return true;
}

}  // namespace bdpt

// DirectIntegrator::render's string dispatch (direct.h:450-461).
extern "C" int32_t bdpt_direct_strategy(const char* name) {
    static const char* names[] = {"area", "solidAngle", "cosineHemisphere", "bsdf", "mis"};
    for (int32_t i = 0; name && i < 5; i++)
        if (std::strcmp(name, names[i]) == 0) return i + 1;
    return 0;
}

extern "C" int bdpt_config_load_toml(const char* toml_path, bdpt_config* out) {
    if (!toml_path || !out) return bdpt::set_error(BDPT_ERR_INVALID, "bdpt_config_load_toml: null argument");
    std::string err;
    if (!bdpt::load_toml_config(toml_path, *out, err)) return bdpt::set_error(BDPT_ERR_INVALID, err);
    return BDPT_OK;
}
