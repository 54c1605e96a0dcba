// events.cpp — translateEventToBinding (pkg/controller/annotator/event.go:118-145):
// the controller's source of the (node, timestamp) pairs K2 counts.
//
//   fmt.Fscanf(strings.NewReader(event.Message), "Successfully assigned %s to %s", &metaKey, &nodeName)
//   namespace, name, err := cache.SplitMetaNamespaceKey(metaKey)
//   Timestamp = event.EventTime.Unix() if event.Count == 0 else event.LastTimestamp.Unix()
//
// The scan restates go1.17 fmt's doScanf/advance for this format: literal runes
// must match; a run of spaces in the format matches one or more spaces of the
// input (or its end); each %s skips spaces (a newline there is an error: Fscanf
// does not treat newlines as spaces), needs at least one rune and reads up to
// the next space; input after the last verb is ignored.  "Space" is Go's
// unicode.IsSpace set (fmt's space table).
#include <cstdint>
#include <cstring>

#include "../../include/crane_dyn.h"

namespace {

struct Scan {
    const unsigned char* s;
    size_t n, i;
    // next rune (code point) and its byte width at i; -1 at the end
    int32_t peek(size_t* w) const {
        if (i >= n) {
            *w = 0;
            return -1;
        }
        const unsigned char c = s[i];
        auto cont = [&](size_t k) { return i + k < n && (s[i + k] & 0xC0) == 0x80; };
        if (c < 0x80) {
            *w = 1;
            return c;
        }
        if ((c & 0xE0) == 0xC0 && cont(1)) {
            const int32_t r = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F);
            if (r >= 0x80) {
                *w = 2;
                return r;
            }
        } else if ((c & 0xF0) == 0xE0 && cont(1) && cont(2)) {
            const int32_t r = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
            if (r >= 0x800 && (r < 0xD800 || r > 0xDFFF)) {
                *w = 3;
                return r;
            }
        } else if ((c & 0xF8) == 0xF0 && cont(1) && cont(2) && cont(3)) {
            const int32_t r =
                ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
            if (r >= 0x10000 && r <= 0x10FFFF) {
                *w = 4;
                return r;
            }
        }
        *w = 1;  // invalid UTF-8: U+FFFD, one byte
        return 0xFFFD;
    }
};

// fmt's isSpace: the unicode.White_Space ranges
bool is_space(int32_t r) {
    return (r >= 0x09 && r <= 0x0D) || r == 0x20 || r == 0x85 || r == 0xA0 || r == 0x1680 ||
           (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 || r == 0x202F || r == 0x205F || r == 0x3000;
}

// a run of (non-newline) spaces in the format: one or more input spaces, or end of input
bool match_space(Scan& sc) {
    size_t w;
    int32_t r = sc.peek(&w);
    if (r == -1) return true;
    if (!is_space(r) || r == '\n') return false;
    while (r != -1 && is_space(r) && r != '\n') {
        sc.i += w;
        r = sc.peek(&w);
    }
    return true;
}

bool match_literal(Scan& sc, const char* lit) {
    for (const char* p = lit; *p; ++p) {
        if (sc.i >= sc.n || sc.s[sc.i] != (unsigned char)*p) return false;  // ASCII literal runes
        ++sc.i;
    }
    return true;
}

// %s: SkipSpace (newline = error), notEOF, then the token up to the next space
bool scan_token(Scan& sc, size_t* start, size_t* len) {
    size_t w;
    int32_t r = sc.peek(&w);
    while (r != -1 && is_space(r)) {
        if (r == '\r' && sc.i + 1 < sc.n && sc.s[sc.i + 1] == '\n') {
            sc.i += 1;
            r = sc.peek(&w);
            continue;
        }
        if (r == '\n') return false;  // "unexpected newline"
        sc.i += w;
        r = sc.peek(&w);
    }
    if (r == -1) return false;  // io.ErrUnexpectedEOF
    *start = sc.i;
    while (r != -1 && !is_space(r)) {
        sc.i += w;
        r = sc.peek(&w);
    }
    *len = sc.i - *start;
    return true;
}

int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}

}  // namespace

extern "C" int crane_translate_event(const char* msg, size_t n, int32_t count, int64_t event_time_ns,
                                     int64_t last_timestamp_ns, const char** node, size_t* node_len,
                                     const char** ns, size_t* ns_len, const char** pod, size_t* pod_len,
                                     int64_t* ts_s) {
    if (!msg && n) return CRANE_E_INVALID;
    Scan sc{reinterpret_cast<const unsigned char*>(msg), n, 0};
    size_t k0 = 0, kl = 0, n0 = 0, nl = 0;
    const bool ok = match_literal(sc, "Successfully") && match_space(sc) && match_literal(sc, "assigned") &&
                    match_space(sc) && scan_token(sc, &k0, &kl) && match_space(sc) && match_literal(sc, "to") &&
                    match_space(sc) && scan_token(sc, &n0, &nl);
    if (!ok) return CRANE_E_PARSE;
    // cache.SplitMetaNamespaceKey: 1 part -> ("", key), 2 parts -> (ns, name), else an error
    const char* key = msg + k0;
    const char* slash = static_cast<const char*>(std::memchr(key, '/', kl));
    size_t nsl = 0, po = 0;
    if (slash) {
        nsl = (size_t)(slash - key);
        po = nsl + 1;
        if (std::memchr(key + po, '/', kl - po)) return CRANE_E_PARSE;
    }
    if (node) *node = msg + n0;
    if (node_len) *node_len = nl;
    if (ns) *ns = key;
    if (ns_len) *ns_len = nsl;
    if (pod) *pod = key + po;
    if (pod_len) *pod_len = kl - po;
    if (ts_s) *ts_s = floor_div(count == 0 ? event_time_ns : last_timestamp_ns, 1000000000LL);
    return CRANE_OK;
}
