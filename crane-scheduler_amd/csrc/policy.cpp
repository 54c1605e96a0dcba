// policy.cpp — strict decoder for DynamicSchedulerPolicy files.
//
// Replaces LoadPolicyFromFile/loadPolicy (pkg/plugins/dynamic/policyfile.go:11-33):
// the reference decodes with the apimachinery UniversalDecoder of a scheme
// built with serializer.EnableStrict (pkg/plugins/apis/policy/scheme/scheme.go:17),
// i.e. YAML -> JSON -> strict json.Unmarshal into v1alpha1.DynamicSchedulerPolicy
// (pkg/plugins/apis/policy/v1alpha1/types.go:9-39), then conversion to the
// internal type (conversion_generated.go).  Consequences restated here:
//   - apiVersion must be scheduler.policy.crane.io/v1alpha1, kind
//     DynamicSchedulerPolicy (register.go:9); unknown or duplicate fields fail;
//   - metav1.Duration fields must be JSON strings accepted by time.ParseDuration;
//   - maxLimitPecent/weight are JSON numbers; count is an integer literal;
//   - a null value leaves the Go zero value.
// Supported syntax: JSON, and the YAML block subset policy files use
// (mappings, sequences, "- key: value" items, comments, plain/quoted
// scalars, empty flow collections [] / {}).
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/crane_dyn.h"

namespace {

struct Node {
    enum Kind { Null, Scalar, Map, Seq } kind = Null;
    std::string text;  // scalar text
    bool quoted = false;
    std::vector<std::pair<std::string, std::unique_ptr<Node>>> map;
    std::vector<std::unique_ptr<Node>> seq;
};

struct ParseError {
    std::string msg;
};

[[noreturn]] void fail(const std::string& m) { throw ParseError{m}; }

// ------------------------------------------------------------------ JSON
struct Json {
    const std::string& s;
    size_t i = 0;
    explicit Json(const std::string& x) : s(x) {}
    void ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
    }
    std::string str() {
        if (s[i] != '"') fail("expected string");
        ++i;
        std::string out;
        while (i < s.size() && s[i] != '"') {
            char c = s[i++];
            if (c == '\\') {
                if (i >= s.size()) fail("bad escape");
                char e = s[i++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (i + 4 > s.size()) fail("bad \\u escape");
                        unsigned v = (unsigned)std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
                        i += 4;
                        if (v < 0x80) out += (char)v;
                        else if (v < 0x800) { out += (char)(0xC0 | (v >> 6)); out += (char)(0x80 | (v & 63)); }
                        else { out += (char)(0xE0 | (v >> 12)); out += (char)(0x80 | ((v >> 6) & 63)); out += (char)(0x80 | (v & 63)); }
                        break;
                    }
                    default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (i >= s.size()) fail("unterminated string");
        ++i;
        return out;
    }
    std::unique_ptr<Node> value() {
        ws();
        if (i >= s.size()) fail("unexpected end of JSON");
        auto n = std::make_unique<Node>();
        char c = s[i];
        if (c == '{') {
            n->kind = Node::Map;
            ++i;
            ws();
            if (s[i] == '}') { ++i; return n; }
            for (;;) {
                ws();
                std::string k = str();
                ws();
                if (s[i] != ':') fail("expected ':'");
                ++i;
                n->map.emplace_back(k, value());
                ws();
                if (s[i] == ',') { ++i; continue; }
                if (s[i] == '}') { ++i; break; }
                fail("expected ',' or '}'");
            }
        } else if (c == '[') {
            n->kind = Node::Seq;
            ++i;
            ws();
            if (s[i] == ']') { ++i; return n; }
            for (;;) {
                n->seq.push_back(value());
                ws();
                if (s[i] == ',') { ++i; continue; }
                if (s[i] == ']') { ++i; break; }
                fail("expected ',' or ']'");
            }
        } else if (c == '"') {
            n->kind = Node::Scalar;
            n->quoted = true;
            n->text = str();
        } else {
            size_t j = i;
            while (j < s.size() && !std::strchr(",]} \t\r\n", s[j])) ++j;
            n->text = s.substr(i, j - i);
            i = j;
            if (n->text == "null") n->kind = Node::Null;
            else n->kind = Node::Scalar;
        }
        return n;
    }
};

// ------------------------------------------------------------------ YAML
struct Line {
    int indent;
    std::string text;
    int no;
};

std::string strip_comment(const std::string& s) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < s.size(); ++i) {
        char c = s[i];
        if (c == '\'' && !dq) sq = !sq;
        else if (c == '"' && !sq) dq = !dq;
        else if (c == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
    }
    return s;
}

std::string rtrim(std::string s) {
    while (!s.empty() && std::isspace((unsigned char)s.back())) s.pop_back();
    return s;
}

std::unique_ptr<Node> yaml_scalar(const std::string& raw, int no) {
    auto n = std::make_unique<Node>();
    std::string t = rtrim(raw);
    size_t a = 0;
    while (a < t.size() && t[a] == ' ') ++a;
    t = t.substr(a);
    if (t.empty() || t == "~" || t == "null" || t == "Null" || t == "NULL") return n;
    if (t == "[]") { n->kind = Node::Seq; return n; }
    if (t == "{}") { n->kind = Node::Map; return n; }
    n->kind = Node::Scalar;
    if (t[0] == '"' || t[0] == '\'') {
        const char q = t[0];
        if (t.size() < 2 || t.back() != q) fail("line " + std::to_string(no) + ": unterminated quoted scalar");
        std::string body = t.substr(1, t.size() - 2);
        if (q == '\'') {
            std::string out;
            for (size_t i = 0; i < body.size(); ++i) {
                out += body[i];
                if (body[i] == '\'' && i + 1 < body.size() && body[i + 1] == '\'') ++i;
            }
            body = out;
        } else {
            std::string js = "\"" + body + "\"";
            Json j(js);
            body = j.str();
        }
        n->text = body;
        n->quoted = true;
        return n;
    }
    if (t[0] == '[' || t[0] == '{') fail("line " + std::to_string(no) + ": flow collections are not supported");
    if (t[0] == '&' || t[0] == '*' || t[0] == '!' || t[0] == '|' || t[0] == '>')
        fail("line " + std::to_string(no) + ": unsupported YAML construct");
    n->text = t;
    return n;
}

// split "key: value" at the first ": " (or trailing ':') outside quotes
bool split_key(const std::string& t, std::string* k, std::string* v) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < t.size(); ++i) {
        char c = t[i];
        if (c == '\'' && !dq) sq = !sq;
        else if (c == '"' && !sq) dq = !dq;
        else if (c == ':' && !sq && !dq && (i + 1 == t.size() || t[i + 1] == ' ')) {
            *k = rtrim(t.substr(0, i));
            *v = i + 1 < t.size() ? t.substr(i + 1) : "";
            if (!k->empty() && (((*k)[0] == '"' && k->back() == '"') || ((*k)[0] == '\'' && k->back() == '\'')))
                *k = k->substr(1, k->size() - 2);
            return true;
        }
    }
    return false;
}

struct Yaml {
    std::vector<Line> L;
    size_t i = 0;

    std::unique_ptr<Node> block(int indent) {
        if (i >= L.size()) return std::make_unique<Node>();
        if (L[i].text == "-" || L[i].text.rfind("- ", 0) == 0) return seq(indent);
        return map(indent);
    }
    std::unique_ptr<Node> seq(int indent) {
        auto n = std::make_unique<Node>();
        n->kind = Node::Seq;
        while (i < L.size() && L[i].indent == indent && (L[i].text == "-" || L[i].text.rfind("- ", 0) == 0)) {
            if (L[i].text == "-") {
                ++i;
                if (i < L.size() && L[i].indent > indent) n->seq.push_back(block(L[i].indent));
                else n->seq.push_back(std::make_unique<Node>());
                continue;
            }
            size_t off = 1;
            while (off < L[i].text.size() && L[i].text[off] == ' ') ++off;
            std::string rest = L[i].text.substr(off);
            std::string k, v;
            if (split_key(rest, &k, &v)) {
                L[i].indent = indent + (int)off;  // the item's mapping starts at the key column
                L[i].text = rest;
                n->seq.push_back(map(L[i].indent));
            } else {
                n->seq.push_back(yaml_scalar(rest, L[i].no));
                ++i;
            }
        }
        if (i < L.size() && L[i].indent > indent) fail("line " + std::to_string(L[i].no) + ": bad indentation");
        return n;
    }
    std::unique_ptr<Node> map(int indent) {
        auto n = std::make_unique<Node>();
        n->kind = Node::Map;
        while (i < L.size() && L[i].indent == indent) {
            std::string k, v;
            if (!split_key(L[i].text, &k, &v)) fail("line " + std::to_string(L[i].no) + ": expected 'key: value'");
            const int no = L[i].no;
            ++i;
            std::string vt = rtrim(v);
            while (!vt.empty() && vt[0] == ' ') vt.erase(0, 1);
            if (vt.empty()) {
                if (i < L.size() && L[i].indent > indent) n->map.emplace_back(k, block(L[i].indent));
                else if (i < L.size() && L[i].indent == indent && (L[i].text == "-" || L[i].text.rfind("- ", 0) == 0))
                    n->map.emplace_back(k, seq(indent));
                else n->map.emplace_back(k, std::make_unique<Node>());
            } else {
                n->map.emplace_back(k, yaml_scalar(vt, no));
                if (i < L.size() && L[i].indent > indent)
                    fail("line " + std::to_string(L[i].no) + ": unexpected indentation");
            }
        }
        if (i < L.size() && L[i].indent > indent) fail("line " + std::to_string(L[i].no) + ": bad indentation");
        return n;
    }
};

std::unique_ptr<Node> parse_doc(const std::string& data) {
    size_t a = 0;
    while (a < data.size() && std::isspace((unsigned char)data[a])) ++a;
    if (a < data.size() && data[a] == '{') {
        Json j(data);
        j.i = a;
        auto n = j.value();
        j.ws();
        if (j.i != data.size()) fail("trailing data after JSON document");
        return n;
    }
    Yaml y;
    std::istringstream in(data);
    std::string line;
    int no = 0;
    bool started = false;
    while (std::getline(in, line)) {
        ++no;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.find('\t') != std::string::npos && line.find_first_not_of(" \t") != std::string::npos &&
            line.find_first_not_of(" ") < line.size() && line[line.find_first_not_of(" ")] == '\t')
            fail("line " + std::to_string(no) + ": tab indentation");
        if (line == "---") {
            if (started) fail("multiple YAML documents");
            continue;
        }
        std::string t = rtrim(strip_comment(line));
        size_t ind = t.find_first_not_of(' ');
        if (ind == std::string::npos) continue;
        started = true;
        y.L.push_back({(int)ind, t.substr(ind), no});
    }
    if (y.L.empty()) fail("empty document");
    auto n = y.block(y.L[0].indent);
    if (y.i != y.L.size()) fail("line " + std::to_string(y.L[y.i].no) + ": unexpected content");
    return n;
}

// ------------------------------------------------------------- decoding
inline bool digit(char c) { return c >= '0' && c <= '9'; }

// go-yaml (via sigs.k8s.io/yaml) resolves a plain scalar matching the YAML
// int/float forms to a JSON number; everything else stays a string.
bool is_yaml_number(const Node& n) {
    if (n.quoted || n.kind != Node::Scalar) return false;
    const std::string& t = n.text;
    if (t == ".inf" || t == "-.inf" || t == "+.inf" || t == ".Inf" || t == "-.Inf" || t == "+.Inf" || t == ".nan" ||
        t == ".NaN" || t == ".NAN")
        return true;
    size_t i = 0;
    if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
    size_t d0 = i;
    while (i < t.size() && (digit(t[i]) || t[i] == '_')) ++i;
    bool mant = i > d0;
    if (i < t.size() && t[i] == '.') {
        ++i;
        size_t f0 = i;
        while (i < t.size() && (digit(t[i]) || t[i] == '_')) ++i;
        mant = mant || i > f0;
    }
    if (!mant) return false;
    if (i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
        ++i;
        if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
        size_t e0 = i;
        while (i < t.size() && digit(t[i])) ++i;
        if (i == e0) return false;
    }
    return i == t.size();
}

bool is_yaml_bool(const Node& n) {
    if (n.quoted || n.kind != Node::Scalar) return false;
    static const char* b[] = {"y", "Y", "yes", "Yes", "YES", "n", "N", "no", "No", "NO", "true", "True", "TRUE",
                              "false", "False", "FALSE", "on", "On", "ON", "off", "Off", "OFF"};
    for (const char* x : b)
        if (n.text == x) return true;
    return false;
}

double to_double(const Node& n, const std::string& field) {
    if (n.kind == Node::Null) return 0.0;
    if (!is_yaml_number(n)) fail(field + ": cannot unmarshal \"" + n.text + "\" into float64");
    const std::string& t = n.text;
    if (t == ".inf" || t == "+.inf" || t == ".Inf" || t == "-.inf" || t == "-.Inf" || t == ".nan" || t == ".NaN")
        fail(field + ": JSON cannot carry " + t);
    std::string c;
    for (char x : t)
        if (x != '_') c += x;
    return std::strtod(c.c_str(), nullptr);
}

int64_t to_int(const Node& n, const std::string& field) {
    if (n.kind == Node::Null) return 0;
    if (n.quoted || n.kind != Node::Scalar) fail(field + ": expected an integer");
    const std::string& t = n.text;
    size_t a = (t[0] == '-' || t[0] == '+') ? 1 : 0;
    if (a >= t.size()) fail(field + ": expected an integer");
    for (size_t i = a; i < t.size(); ++i)
        if (!std::isdigit((unsigned char)t[i])) fail(field + ": cannot unmarshal number " + t + " into int");
    errno = 0;
    long long v = std::strtoll(t.c_str(), nullptr, 10);
    if (errno == ERANGE) fail(field + ": integer out of range");
    return v;
}

}  // namespace

bool crane_go_parse_duration(const char* s, size_t n, int64_t* out_ns);  // below

namespace {

int64_t to_duration(const Node& n, const std::string& field) {
    if (n.kind == Node::Null) return 0;
    if (n.kind != Node::Scalar) fail(field + ": expected a duration string");
    // sigs.k8s.io/yaml turns plain numbers into JSON numbers; metav1.Duration
    // only unmarshals from a JSON string.
    if (!n.quoted && (is_yaml_number(n) || is_yaml_bool(n))) fail(field + ": cannot unmarshal " + n.text + " into Duration");
    int64_t d;
    if (!crane_go_parse_duration(n.text.c_str(), n.text.size(), &d)) fail(field + ": time: invalid duration \"" + n.text + "\"");
    return d;
}

std::string to_string(const Node& n, const std::string& field) {
    if (n.kind == Node::Null) return "";
    if (n.kind != Node::Scalar) fail(field + ": expected a string");
    if (!n.quoted && (is_yaml_number(n) || is_yaml_bool(n)))
        fail(field + ": cannot unmarshal " + n.text + " into string");
    return n.text;
}

template <typename F>
void fields(const Node& n, const std::string& where, const std::vector<std::string>& allowed, F&& f) {
    if (n.kind == Node::Null) return;
    if (n.kind != Node::Map) fail(where + ": expected an object");
    std::vector<std::string> seen;
    for (const auto& kv : n.map) {
        bool ok = false;
        for (const auto& a : allowed) ok |= a == kv.first;
        if (!ok) fail("strict decoding error: unknown field \"" + where + "." + kv.first + "\"");
        for (const auto& s : seen)
            if (s == kv.first) fail("strict decoding error: duplicate field \"" + where + "." + kv.first + "\"");
        seen.push_back(kv.first);
        f(kv.first, *kv.second);
    }
}

template <typename F>
void items(const Node& n, const std::string& where, F&& f) {
    if (n.kind == Node::Null) return;
    if (n.kind != Node::Seq) fail(where + ": expected a list");
    for (size_t i = 0; i < n.seq.size(); ++i) f(*n.seq[i], where + "[" + std::to_string(i) + "]");
}

}  // namespace

// time.ParseDuration (go1.17 time/format.go)
bool crane_go_parse_duration(const char* s, size_t n, int64_t* out_ns) {
    const uint64_t B63 = 1ULL << 63;
    uint64_t d = 0;
    bool neg = false;
    size_t i = 0;
    if (n > 0 && (s[0] == '-' || s[0] == '+')) { neg = s[0] == '-'; i = 1; }
    if (n - i == 1 && s[i] == '0') { *out_ns = 0; return true; }
    if (i == n) return false;
    while (i < n) {
        uint64_t v = 0, f = 0;
        double scale = 1;
        if (!(s[i] == '.' || digit(s[i]))) return false;
        const size_t st = i;
        for (; i < n && digit(s[i]); ++i) {
            if (v > B63 / 10) return false;
            v = v * 10 + (uint64_t)(s[i] - '0');
            if (v > B63) return false;
        }
        const bool pre = i != st;
        bool post = false;
        if (i < n && s[i] == '.') {
            ++i;
            const size_t fs = i;
            bool ovf = false;
            for (; i < n && digit(s[i]); ++i) {
                if (ovf) continue;
                if (f > (B63 - 1) / 10) { ovf = true; continue; }
                const uint64_t y = f * 10 + (uint64_t)(s[i] - '0');
                if (y > B63) { ovf = true; continue; }
                f = y;
                scale *= 10;
            }
            post = i != fs;
        }
        if (!pre && !post) return false;
        const size_t us = i;
        while (i < n && !(s[i] == '.' || digit(s[i]))) ++i;
        const std::string u(s + us, i - us);
        uint64_t unit;
        if (u == "ns") unit = 1;
        else if (u == "us" || u == "\xc2\xb5s" || u == "\xce\xbcs") unit = 1000;
        else if (u == "ms") unit = 1000000;
        else if (u == "s") unit = 1000000000ULL;
        else if (u == "m") unit = 60000000000ULL;
        else if (u == "h") unit = 3600000000000ULL;
        else return false;
        if (v > B63 / unit) return false;
        v *= unit;
        if (f > 0) {
            v += (uint64_t)((double)f * ((double)unit / scale));
            if (v > B63) return false;
        }
        d += v;
        if (d > B63) return false;
    }
    if (neg) { *out_ns = (int64_t)(0 - d); return true; }
    if (d > B63 - 1) return false;
    *out_ns = (int64_t)d;
    return true;
}

struct crane_policy_doc {
    std::vector<std::string> sync_name, pred_name, prio_name;
    std::vector<const char*> sync_p, pred_p, prio_p;
    std::vector<int64_t> sync_period, hot_tr, hot_count;
    std::vector<double> pred_limit, prio_weight;
    crane_policy view{};
    void finish() {
        sync_p.clear(); pred_p.clear(); prio_p.clear();
        for (auto& s : sync_name) sync_p.push_back(s.c_str());
        for (auto& s : pred_name) pred_p.push_back(s.c_str());
        for (auto& s : prio_name) prio_p.push_back(s.c_str());
        view.n_sync = (int32_t)sync_name.size();
        view.sync_name = sync_p.data();
        view.sync_period_ns = sync_period.data();
        view.n_pred = (int32_t)pred_name.size();
        view.pred_name = pred_p.data();
        view.pred_limit = pred_limit.data();
        view.n_prio = (int32_t)prio_name.size();
        view.prio_name = prio_p.data();
        view.prio_weight = prio_weight.data();
        view.n_hot = (int32_t)hot_tr.size();
        view.hot_tr_ns = hot_tr.data();
        view.hot_count = hot_count.data();
    }
};

static void decode(const Node& root, crane_policy_doc* d) {
    std::string api, kind;
    const Node* spec = nullptr;
    fields(root, "", {"apiVersion", "kind", "spec"}, [&](const std::string& k, const Node& v) {
        if (k == "apiVersion") api = to_string(v, "apiVersion");
        else if (k == "kind") kind = to_string(v, "kind");
        else spec = &v;
    });
    if (kind.empty()) fail("Object 'Kind' is missing");
    if (api.empty()) fail("Object 'apiVersion' is missing");
    if (api != "scheduler.policy.crane.io/v1alpha1" || kind != "DynamicSchedulerPolicy")
        fail("no kind \"" + kind + "\" is registered for version \"" + api + "\"");
    if (!spec) return;
    fields(*spec, "spec", {"syncPolicy", "predicate", "priority", "hotValue"}, [&](const std::string& k, const Node& v) {
        if (k == "syncPolicy")
            items(v, "spec.syncPolicy", [&](const Node& it, const std::string& w) {
                std::string name;
                int64_t period = 0;
                fields(it, w, {"name", "period"}, [&](const std::string& f, const Node& x) {
                    if (f == "name") name = to_string(x, w + ".name");
                    else period = to_duration(x, w + ".period");
                });
                d->sync_name.push_back(name);
                d->sync_period.push_back(period);
            });
        else if (k == "predicate")
            items(v, "spec.predicate", [&](const Node& it, const std::string& w) {
                std::string name;
                double lim = 0;
                fields(it, w, {"name", "maxLimitPecent"}, [&](const std::string& f, const Node& x) {
                    if (f == "name") name = to_string(x, w + ".name");
                    else lim = to_double(x, w + ".maxLimitPecent");
                });
                d->pred_name.push_back(name);
                d->pred_limit.push_back(lim);
            });
        else if (k == "priority")
            items(v, "spec.priority", [&](const Node& it, const std::string& w) {
                std::string name;
                double wt = 0;
                fields(it, w, {"name", "weight"}, [&](const std::string& f, const Node& x) {
                    if (f == "name") name = to_string(x, w + ".name");
                    else wt = to_double(x, w + ".weight");
                });
                d->prio_name.push_back(name);
                d->prio_weight.push_back(wt);
            });
        else
            items(v, "spec.hotValue", [&](const Node& it, const std::string& w) {
                int64_t tr = 0, c = 0;
                fields(it, w, {"timeRange", "count"}, [&](const std::string& f, const Node& x) {
                    if (f == "timeRange") tr = to_duration(x, w + ".timeRange");
                    else c = to_int(x, w + ".count");
                });
                d->hot_tr.push_back(tr);
                d->hot_count.push_back(c);
            });
    });
}

extern "C" {

int crane_policy_load_bytes(const char* data, size_t n, crane_policy_doc** out, char* err, size_t errcap) {
    if (!out) return CRANE_E_INVALID;
    *out = nullptr;
    auto d = std::make_unique<crane_policy_doc>();
    try {
        auto root = parse_doc(std::string(data ? data : "", data ? n : 0));
        decode(*root, d.get());
    } catch (const ParseError& e) {
        if (err && errcap) std::snprintf(err, errcap, "%s", e.msg.c_str());
        return CRANE_E_PARSE;
    }
    d->finish();
    *out = d.release();
    return CRANE_OK;
}

int crane_policy_load_file(const char* path, crane_policy_doc** out, char* err, size_t errcap) {
    if (!out) return CRANE_E_INVALID;
    *out = nullptr;
    std::ifstream f(path ? path : "", std::ios::binary);
    if (!f) {
        if (err && errcap) std::snprintf(err, errcap, "open %s: no such file or directory", path ? path : "");
        return CRANE_E_IO;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string s = ss.str();
    return crane_policy_load_bytes(s.data(), s.size(), out, err, errcap);
}

const crane_policy* crane_policy_view(const crane_policy_doc* d) { return d ? &d->view : nullptr; }

void crane_policy_free(crane_policy_doc* d) { delete d; }

}  // extern "C"
