/*
 * crane_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of crane-scheduler's Dynamic plugin Filter + Score hot path
 * and of the controller's hot-value producer.  Every function cites the
 * reference file:line it follows (paths relative to /root/reference).
 *
 * Parity: UNPINNED BY THE REFERENCE — the reference has no tests, fixtures or
 * golden vectors for this path (its only tests cover the NodeResourceTopology
 * plugin) and it is Go code whose toolchain/modules are absent here, so it
 * cannot be run.  This restatement is pinned by hand-derived known-answer
 * tests (tests/golden/kats.json) and a golden cluster computed by an
 * independent pure-Python restatement (tests/golden/make_golden.py).
 *
 * Build: see oracle/Makefile (-O2 -ffp-contract=off, no -ffast-math: Go on
 * amd64 never contracts a*b+c into an FMA, so neither may we).
 */
#define _GNU_SOURCE
#include "crane_oracle.h"

#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* stats.go:18-26 */
#define MIN_TIMESTAMP_STR_LENGTH 5
#define NODE_HOT_VALUE "node_hot_value"
#define HOT_VALUE_ACTIVE_NS (5LL * 60 * 1000000000LL)
#define EXTRA_ACTIVE_NS (5LL * 60 * 1000000000LL)
/* upstream k8s v1.23.3 framework.MaxNodeScore / MinNodeScore */
#define MAX_NODE_SCORE 100
#define MIN_NODE_SCORE 0

/* ------------------------------------------------------------------ */
/* Go: int(float64) on amd64 — CVTTSD2SQ yields 0x8000000000000000 for NaN
 * and out-of-range inputs (stats.go:135, plugins.go:91).                 */
int64_t or_go_f64_to_int(double x) {
    if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
    return (int64_t)x;
}

/* Go: int64(d.Seconds()) where Seconds() = float64(d/1e9) + float64(d%1e9)/1e9
 * (binding.go:85). */
int64_t or_go_duration_seconds_trunc(int64_t d) {
    int64_t sec = d / 1000000000LL, nsec = d % 1000000000LL;
    double s = (double)sec + (double)nsec / 1e9;
    return or_go_f64_to_int(s);
}

/* ------------------------------------------------------------------ */
/* strconv.ParseFloat(s, 64) grammar (go1.17 strconv/atof.go: special,
 * readFloat, underscoreOK); the value itself is the correctly rounded
 * conversion, which glibc strtod also computes.                          */
static int lower(int c) { return c | 0x20; }

static int prefix_ci(const char *s, int64_t n, const char *word) {
    int64_t i = 0;
    while (i < n && word[i] && lower((unsigned char)s[i]) == word[i]) i++;
    return (int)i;
}

static int underscore_ok(const char *s, int64_t n) {
    char saw = '^';
    int64_t i = 0;
    if (n >= 1 && (s[0] == '-' || s[0] == '+')) { s++; n--; }
    int hex = 0;
    if (n >= 2 && s[0] == '0' && (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
        i = 2; saw = '0'; hex = lower(s[1]) == 'x';
    }
    for (; i < n; i++) {
        char c = s[i];
        if ((c >= '0' && c <= '9') || (hex && lower(c) >= 'a' && lower(c) <= 'f')) { saw = '0'; continue; }
        if (c == '_') { if (saw != '0') return 0; saw = '_'; continue; }
        if (saw == '_') return 0;
        saw = '!';
    }
    return saw != '_';
}

int or_go_parse_float(const char *s, int64_t n, double *out) {
    *out = 0;
    if (n <= 0) return 1;
    /* special(): optional sign + "inf"/"infinity", or unsigned "nan". */
    {
        int64_t i = 0; double sign = 1;
        int ok = 0, cons = 0;
        if (s[0] == '+' || s[0] == '-') {
            if (s[0] == '-') sign = -1;
            i = 1;
            int k = prefix_ci(s + 1, n - 1, "infinity");
            if (k > 3 && k < 8) k = 3;
            if (k == 3 || k == 8) { ok = 1; cons = 1 + k; }
        } else if (lower(s[0]) == 'i') {
            int k = prefix_ci(s, n, "infinity");
            if (k > 3 && k < 8) k = 3;
            if (k == 3 || k == 8) { ok = 1; cons = k; }
        } else if (lower(s[0]) == 'n') {
            if (prefix_ci(s, n, "nan") == 3) { ok = 2; cons = 3; }
        }
        (void)i;
        if (ok) {
            if (cons != n) return 1;
            *out = ok == 2 ? NAN : sign * INFINITY;
            return 0;
        }
    }
    /* readFloat() */
    int64_t i = 0;
    int neg = 0, hex = 0, underscores = 0, sawdot = 0, sawdigits = 0;
    if (s[i] == '+') i++;
    else if (s[i] == '-') { neg = 1; i++; }
    (void)neg;
    int base = 10;
    char exp_char = 'e';
    if (i + 2 < n && s[i] == '0' && lower(s[i + 1]) == 'x') { base = 16; i += 2; exp_char = 'p'; hex = 1; }
    for (; i < n; i++) {
        char c = s[i];
        if (c == '_') { underscores = 1; continue; }
        if (c == '.') { if (sawdot) break; sawdot = 1; continue; }
        if (c >= '0' && c <= '9') { sawdigits = 1; continue; }
        if (base == 16 && lower(c) >= 'a' && lower(c) <= 'f') { sawdigits = 1; continue; }
        break;
    }
    if (!sawdigits) return 1;
    if (i < n && lower(s[i]) == exp_char) {
        i++;
        if (i >= n) return 1;
        if (s[i] == '+' || s[i] == '-') i++;
        if (i >= n || s[i] < '0' || s[i] > '9') return 1;
        for (; i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); i++)
            if (s[i] == '_') underscores = 1;
    } else if (base == 16) {
        return 1; /* hex mantissa must have a 'p' exponent */
    }
    if (underscores && !underscore_ok(s, i)) return 1;
    if (i != n) return 1; /* ParseFloat: trailing bytes are a syntax error */
    /* value: strip underscores, correctly rounded conversion */
    char stackbuf[128];
    char *buf = n < (int64_t)sizeof stackbuf ? stackbuf : (char *)malloc((size_t)n + 1);
    int64_t m = 0;
    for (int64_t j = 0; j < n; j++) if (s[j] != '_') buf[m++] = s[j];
    buf[m] = 0;
    errno = 0;
    char *end = NULL;
    double v = strtod(buf, &end);
    int bad = (end != buf + m);
    if (buf != stackbuf) free(buf);
    if (bad) return 1;
    (void)hex;
    *out = v;
    if (isinf(v)) return 2; /* Go: ErrRange on overflow (returns ±Inf + error) */
    return 0;                /* underflow to 0/denormal is not an error in Go */
}

/* ------------------------------------------------------------------ */
/* time.ParseInLocation(utils.TimeFormat = "2006-01-02T15:04:05Z", s, loc)
 * (stats.go:37, utils.go:11).  Layout chunks (go1.17 time/format.go):
 * stdLongYear, '-', stdZeroMonth, '-', stdZeroDay, 'T', stdHour, ':',
 * stdZeroMinute, ':', stdZeroSecond (+ optional .fraction), literal 'Z'.
 * loc is a fixed UTC offset (Asia/Shanghai is UTC+8 since 1991).        */
static int is_digit(const char *s, int64_t n, int64_t i) { return i < n && s[i] >= '0' && s[i] <= '9'; }

/* getnum(value, fixed) */
static int getnum(const char *s, int64_t n, int64_t *pos, int fixed, int *out) {
    int64_t i = *pos;
    if (!is_digit(s, n, i)) return -1;
    if (!is_digit(s, n, i + 1)) {
        if (fixed) return -1;
        *out = s[i] - '0'; *pos = i + 1; return 0;
    }
    *out = (s[i] - '0') * 10 + (s[i + 1] - '0');
    *pos = i + 2;
    return 0;
}

static int lit(const char *s, int64_t n, int64_t *pos, char c) {
    if (*pos >= n || s[*pos] != c) return -1;
    (*pos)++;
    return 0;
}

static int is_leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
static int days_in(int m, int64_t y) {
    static const int d[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    return m == 2 && is_leap(y) ? 29 : d[m - 1];
}
/* days since 1970-01-01 of a proleptic Gregorian civil date */
static int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    int64_t era = (y >= 0 ? y : y - 399) / 400;
    int64_t yoe = y - era * 400;
    int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

int or_go_parse_time(const char *s, int64_t n, int64_t tz_offset_s, int64_t *out_ns) {
    int64_t p = 0;
    int year = 0, month, day, hour, min, sec;
    int64_t nsec = 0;
    /* stdLongYear: 4 bytes, first a digit, atoi() of all four */
    if (n < 4 || !is_digit(s, n, 0)) return -1;
    for (int k = 0; k < 4; k++) {
        if (!is_digit(s, n, k)) return -1;
        year = year * 10 + (s[k] - '0');
    }
    p = 4;
    if (lit(s, n, &p, '-')) return -1;
    if (getnum(s, n, &p, 1, &month)) return -1;
    if (month <= 0 || month > 12) return -2;
    if (lit(s, n, &p, '-')) return -1;
    if (getnum(s, n, &p, 1, &day)) return -1;
    if (lit(s, n, &p, 'T')) return -1;
    if (getnum(s, n, &p, 0, &hour)) return -1;
    if (hour < 0 || hour >= 24) return -2;
    if (lit(s, n, &p, ':')) return -1;
    if (getnum(s, n, &p, 1, &min)) return -1;
    if (min < 0 || min >= 60) return -2;
    if (lit(s, n, &p, ':')) return -1;
    if (getnum(s, n, &p, 1, &sec)) return -1;
    if (sec < 0 || sec >= 60) return -2;
    /* fractional second present in the value but not in the layout */
    if (n - p >= 2 && s[p] == '.' && is_digit(s, n, p + 1)) {
        int64_t q = p + 2;
        while (q < n && is_digit(s, n, q)) q++;
        int64_t nbytes = q - p;
        int64_t lim = nbytes > 10 ? 10 : nbytes;
        int64_t ns = 0;
        for (int64_t k = p + 1; k < p + lim; k++) ns = ns * 10 + (s[k] - '0');
        for (int64_t k = 0; k < 10 - lim; k++) ns *= 10;
        nsec = ns;
        p = q;
    }
    if (lit(s, n, &p, 'Z')) return -1;
    if (p != n) return -1; /* extra text */
    if (day < 1 || day > days_in(month, year)) return -2;
    int64_t days = days_from_civil(year, month, day);
    /* int64 ns covers 1678..2262; Go's Time covers more.  Saturate so the
     * ordering (stale long ago / fresh far in the future) is preserved. */
    __int128 t = ((__int128)days * 86400 + hour * 3600 + min * 60 + sec - tz_offset_s) * 1000000000 + nsec;
    const __int128 lo = (__int128)INT64_MIN / 2, hi = (__int128)INT64_MAX / 2;
    if (t < lo) t = lo;
    if (t > hi) t = hi;
    *out_ns = (int64_t)t;
    return 0;
}

/* ------------------------------------------------------------------ */
/* time.ParseDuration (go1.17 time/format.go) for metav1.Duration fields. */
int or_go_parse_duration(const char *s, int64_t n, int64_t *out_ns) {
    const uint64_t B63 = 1ULL << 63;
    uint64_t d = 0;
    int neg = 0;
    int64_t i = 0;
    if (n > 0 && (s[0] == '-' || s[0] == '+')) { neg = s[0] == '-'; i = 1; }
    if (n - i == 1 && s[i] == '0') { *out_ns = 0; return 0; }
    if (i == n) return -1;
    while (i < n) {
        uint64_t v = 0, f = 0;
        double scale = 1;
        if (!(s[i] == '.' || (s[i] >= '0' && s[i] <= '9'))) return -1;
        int64_t st = i;
        for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
            if (v > B63 / 10) return -1;
            v = v * 10 + (uint64_t)(s[i] - '0');
            if (v > B63) return -1;
        }
        int pre = i != st, post = 0;
        if (i < n && s[i] == '.') {
            i++;
            int64_t fs = i;
            int ovf = 0;
            for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
                if (ovf) continue;
                if (f > (B63 - 1) / 10) { ovf = 1; continue; }
                uint64_t y = f * 10 + (uint64_t)(s[i] - '0');
                if (y > B63) { ovf = 1; continue; }
                f = y;
                scale *= 10;
            }
            post = i != fs;
        }
        if (!pre && !post) return -1;
        int64_t us = i;
        for (; i < n; i++) if (s[i] == '.' || (s[i] >= '0' && s[i] <= '9')) break;
        int64_t ul = i - us;
        if (ul == 0) return -1;
        const char *u = s + us;
        uint64_t unit;
        if (ul == 2 && !memcmp(u, "ns", 2)) unit = 1;
        else if (ul == 2 && !memcmp(u, "us", 2)) unit = 1000;
        else if (ul == 3 && !memcmp(u, "\xc2\xb5s", 3)) unit = 1000;
        else if (ul == 3 && !memcmp(u, "\xce\xbcs", 3)) unit = 1000;
        else if (ul == 2 && !memcmp(u, "ms", 2)) unit = 1000000;
        else if (ul == 1 && u[0] == 's') unit = 1000000000ULL;
        else if (ul == 1 && u[0] == 'm') unit = 60000000000ULL;
        else if (ul == 1 && u[0] == 'h') unit = 3600000000000ULL;
        else return -1;
        if (v > B63 / unit) return -1;
        v *= unit;
        if (f > 0) {
            v += (uint64_t)((double)f * ((double)unit / scale));
            if (v > B63) return -1;
        }
        d += v;
        if (d > B63) return -1;
    }
    if (neg) { *out_ns = (int64_t)(0 - d); return 0; }
    if (d > B63 - 1) return -1;
    *out_ns = (int64_t)d;
    return 0;
}

/* ------------------------------------------------------------------ */
/* getActiveDuration (stats.go:140-150) */
int or_active_duration(const or_policy *pol, const char *name, int64_t *dur_ns) {
    for (int32_t i = 0; i < pol->n_sync; i++) {
        if (strcmp(pol->sync_name[i], name) == 0 && pol->sync_period_ns[i] != 0) {
            *dur_ns = pol->sync_period_ns[i] + EXTRA_ACTIVE_NS;
            return 0;
        }
    }
    *dur_ns = 0;
    return -1;
}

/* inActivePeriod's freshness test (stats.go:42-48): now.Before(ts + dur). */
static int fresh(int64_t ts_ns, int64_t dur_ns, int64_t now_ns) {
    __int128 exp = (__int128)ts_ns + dur_ns;
    return (__int128)now_ns < exp;
}

/* Split "<float>,<time>" — strings.Split(v, ",") must give exactly 2 parts
 * (stats.go:57-60); then the time parse (stats.go:31-40) and ParseFloat
 * (stats.go:66-69).  Time-independent errors -> ok = 0. */
void or_parse_annotation(const char *s, int64_t n, int64_t tz, uint8_t *ok, double *val, int64_t *ts_ns) {
    *ok = 0; *val = 0; *ts_ns = 0;
    int64_t comma = -1, ncomma = 0;
    for (int64_t i = 0; i < n; i++) if (s[i] == ',') { ncomma++; if (comma < 0) comma = i; }
    if (ncomma != 1) return;
    const char *t = s + comma + 1;
    int64_t tn = n - comma - 1;
    if (tn < MIN_TIMESTAMP_STR_LENGTH) return;
    if (or_go_parse_time(t, tn, tz, ts_ns)) return;
    double v;
    if (or_go_parse_float(s, comma, &v)) return;
    *val = v;
    *ok = 1;
}

/* ------------------------------------------------------------------ */
/* Evaluation core, generic over how getResourceUsage reads an annotation. */
typedef struct {
    /* string mode */
    const int64_t *anno_off;
    const char *const *keys;
    const char *const *vals;
    int64_t tz;
    /* soa mode */
    const uint8_t *ok;
    const double *val;
    const int64_t *ts;
    const uint8_t *hv_ok;
    const double *hv;
    const int64_t *hv_ts;
    int64_t N;
    const int32_t *pred_row; /* policy entry -> SoA row (-1 = key absent) */
    const int32_t *prio_row;
    int soa;
} usage_src;

/* getResourceUsage (stats.go:51-76): 0 ok (*u set), -1 error. row = SoA
 * row index (or -2 for the hot-value row), name = annotation key. */
static int get_usage(const usage_src *src, int64_t node, const char *name, int32_t row,
                     int64_t dur_ns, int64_t now_ns, double *u) {
    uint8_t ok;
    double v;
    int64_t ts;
    if (src->soa) {
        if (row == -2) { ok = src->hv_ok[node]; v = src->hv[node]; ts = src->hv_ts[node]; }
        else if (row < 0) return -1; /* key not found */
        else {
            size_t ix = (size_t)row * (size_t)src->N + (size_t)node;
            ok = src->ok[ix]; v = src->val[ix]; ts = src->ts[ix];
        }
        if (!ok) return -1;
    } else {
        const char *sv = NULL;
        for (int64_t j = src->anno_off[node]; j < src->anno_off[node + 1]; j++)
            if (strcmp(src->keys[j], name) == 0) { sv = src->vals[j]; break; }
        if (!sv) return -1; /* stats.go:52-55 */
        or_parse_annotation(sv, (int64_t)strlen(sv), src->tz, &ok, &v, &ts);
        if (!ok) return -1;
    }
    if (!fresh(ts, dur_ns, now_ns)) return -1; /* stats.go:62-64 */
    if (v < 0) return -1;                       /* stats.go:71-73 (NaN passes) */
    *u = v;
    return 0;
}

/* isOverLoad (stats.go:94-112) */
static int is_overload(const or_policy *pol, const usage_src *src, int64_t node, int32_t k,
                       int64_t dur, int64_t now) {
    double u;
    if (get_usage(src, node, pol->pred_name[k], src->pred_row ? src->pred_row[k] : -1, dur, now, &u)) return 0;
    if (pol->pred_limit[k] == 0) return 0;
    return u > pol->pred_limit[k];
}

/* DynamicScheduler.Filter (plugins.go:39-69): -1 Success, else index of the
 * first overloaded predicate (Unschedulable). */
static int8_t filter_one(const or_policy *pol, const usage_src *src, int64_t node, int64_t now, int ds) {
    if (ds) return -1; /* plugins.go:41-43 */
    for (int32_t k = 0; k < pol->n_pred; k++) {
        int64_t dur;
        if (or_active_duration(pol, pol->pred_name[k], &dur) || dur == 0) continue; /* :56-61 */
        if (is_overload(pol, src, node, k, dur, now)) return (int8_t)k;            /* :63-65 */
    }
    return -1;
}

/* getNodeScore (stats.go:114-138) with getScore (stats.go:78-92). */
static int64_t node_score(const or_policy *pol, const usage_src *src, int64_t node, int64_t now) {
    if (pol->n_prio == 0) return 0;
    double score = 0, weight = 0;
    for (int32_t k = 0; k < pol->n_prio; k++) {
        double ps = 0, u;
        int64_t dur;
        if (!(or_active_duration(pol, pol->prio_name[k], &dur) || dur == 0)) {
            if (!get_usage(src, node, pol->prio_name[k], src->prio_row ? src->prio_row[k] : -1, dur, now, &u)) {
                ps = (1. - u) * pol->prio_weight[k];
                ps = ps * (double)MAX_NODE_SCORE;
            }
        }
        weight += pol->prio_weight[k];
        score += ps;
    }
    return or_go_f64_to_int(score / weight);
}

/* getNodeHotValue (stats.go:152-166) */
static double node_hot_value(const usage_src *src, int64_t node, int64_t now) {
    double hv;
    if (get_usage(src, node, NODE_HOT_VALUE, -2, HOT_VALUE_ACTIVE_NS, now, &hv)) return 0;
    return hv;
}

/* DynamicScheduler.Score (plugins.go:73-98) */
static int64_t score_one(const or_policy *pol, const usage_src *src, int64_t node, int64_t now) {
    int64_t s = node_score(pol, src, node, now);
    double hv = node_hot_value(src, node, now);
    /* score - int(hotValue*10): Go int64 arithmetic wraps */
    s = (int64_t)((uint64_t)s - (uint64_t)or_go_f64_to_int(hv * 10));
    if (s < MIN_NODE_SCORE) s = MIN_NODE_SCORE; /* utils.NormalizeScore utils.go:58-68 */
    if (s > MAX_NODE_SCORE) s = MAX_NODE_SCORE;
    return s;
}

typedef struct {
    const or_policy *pol;
    const usage_src *src;
    int64_t N, p0, p1;
    const int64_t *now;
    const uint8_t *ds;
    int8_t *ff;
    int64_t *score;
    int64_t *chosen;
} eval_job;

static void *eval_worker(void *arg) {
    eval_job *j = (eval_job *)arg;
    for (int64_t p = j->p0; p < j->p1; p++) {
        int64_t best = -1, best_s = -1;
        int ds = j->ds ? j->ds[p] : 0;
        for (int64_t n = 0; n < j->N; n++) {
            int8_t f = filter_one(j->pol, j->src, n, j->now[p], ds);
            int need_score = j->score || (f < 0 && j->chosen);
            int64_t s = need_score ? score_one(j->pol, j->src, n, j->now[p]) : 0;
            if (j->ff) j->ff[p * j->N + n] = f;
            if (j->score) j->score[p * j->N + n] = s;
            if (f < 0 && s > best_s) { best_s = s; best = n; } /* selectHost, lowest index wins */
        }
        if (j->chosen) j->chosen[p] = best;
    }
    return NULL;
}

static int run_eval(const or_policy *pol, const usage_src *src, int64_t N, int64_t P,
                    const int64_t *now, const uint8_t *ds, int32_t nt,
                    int8_t *ff, int64_t *score, int64_t *chosen) {
    if (nt < 1) nt = 1;
    if (nt > P) nt = (int32_t)(P > 0 ? P : 1);
    eval_job *jobs = (eval_job *)calloc((size_t)nt, sizeof(eval_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nt, sizeof(pthread_t));
    for (int32_t t = 0; t < nt; t++) {
        jobs[t] = (eval_job){pol, src, N, P * t / nt, P * (t + 1) / nt, now, ds, ff, score, chosen};
        if (nt == 1) eval_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, eval_worker, &jobs[t]);
    }
    if (nt > 1) for (int32_t t = 0; t < nt; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    return 0;
}

int or_eval_strings(const or_policy *pol, int64_t N, const int64_t *anno_off,
                    const char *const *keys, const char *const *vals,
                    int64_t P, const int64_t *now_ns, const uint8_t *pod_ds,
                    int64_t tz, int32_t nt, int8_t *ff, int64_t *score, int64_t *chosen) {
    usage_src src;
    memset(&src, 0, sizeof src);
    src.anno_off = anno_off; src.keys = keys; src.vals = vals; src.tz = tz; src.N = N;
    return run_eval(pol, &src, N, P, now_ns, pod_ds, nt, ff, score, chosen);
}

static int32_t *map_rows(int32_t n, const char *const *names, int32_t K, const char *const *key_names) {
    int32_t *r = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (int32_t i = 0; i < n; i++) {
        r[i] = -1;
        for (int32_t k = 0; k < K; k++) if (strcmp(names[i], key_names[k]) == 0) { r[i] = k; break; }
    }
    return r;
}

int or_eval_soa(const or_policy *pol, int32_t K, const char *const *key_names,
                int64_t N, const uint8_t *ok, const double *val, const int64_t *ts,
                const uint8_t *hv_ok, const double *hv, const int64_t *hv_ts,
                int64_t P, const int64_t *now_ns, const uint8_t *pod_ds,
                int32_t nt, int8_t *ff, int64_t *score, int64_t *chosen) {
    usage_src src;
    memset(&src, 0, sizeof src);
    src.soa = 1; src.ok = ok; src.val = val; src.ts = ts; src.N = N;
    src.hv_ok = hv_ok; src.hv = hv; src.hv_ts = hv_ts;
    int32_t *pr = map_rows(pol->n_pred, pol->pred_name, K, key_names);
    int32_t *qr = map_rows(pol->n_prio, pol->prio_name, K, key_names);
    src.pred_row = pr; src.prio_row = qr;
    int rc = run_eval(pol, &src, N, P, now_ns, pod_ds, nt, ff, score, chosen);
    free(pr);
    free(qr);
    return rc;
}

/* ------------------------------------------------------------------ */
/* GetLastNodeBindingCount (binding.go:81-97) for every node at once, and
 * annotateNodeHotValue (node.go:113-121): value += count / p.Count.      */
int or_hot_values(const or_policy *pol, int64_t B, const int32_t *b_node, const int64_t *b_ts,
                  int64_t N, int64_t now_unix, int64_t *cnt, int64_t *hv) {
    int32_t W = pol->n_hot;
    for (int32_t w = 0; w < W; w++) if (pol->hot_count[w] == 0) return -1;
    int64_t *c = cnt ? cnt : (int64_t *)calloc((size_t)(W > 0 ? W : 1) * (size_t)N, sizeof(int64_t));
    if (cnt) memset(cnt, 0, sizeof(int64_t) * (size_t)W * (size_t)N);
    for (int32_t w = 0; w < W; w++) {
        int64_t timeline = now_unix - or_go_duration_seconds_trunc(pol->hot_tr_ns[w]);
        for (int64_t b = 0; b < B; b++) {
            int32_t nd = b_node[b];
            if (nd < 0 || nd >= N) continue;
            if (b_ts[b] > timeline) c[(size_t)w * (size_t)N + (size_t)nd]++;
        }
    }
    for (int64_t n = 0; n < N; n++) {
        int64_t v = 0;
        for (int32_t w = 0; w < W; w++) v += c[(size_t)w * (size_t)N + (size_t)n] / pol->hot_count[w];
        hv[n] = v;
    }
    if (!cnt) free(c);
    return 0;
}

/* ------------------------------------------------------------------ */
int or_greedy(const or_policy *pol, int32_t K, const char *const *key_names,
              int64_t N, const uint8_t *ok, const double *val, const int64_t *ts,
              int64_t B, const int32_t *b_node, const int64_t *b_ts,
              int64_t P, int64_t now_ns, const uint8_t *pod_ds, int64_t *chosen) {
    int32_t W = pol->n_hot;
    int64_t now_unix = now_ns >= 0 ? now_ns / 1000000000LL : -((-now_ns + 999999999LL) / 1000000000LL);
    int64_t *cnt = (int64_t *)calloc((size_t)(W > 0 ? W : 1) * (size_t)N, sizeof(int64_t));
    int64_t *hvi = (int64_t *)calloc((size_t)N, sizeof(int64_t));
    if (or_hot_values(pol, B, b_node, b_ts, N, now_unix, cnt, hvi)) { free(cnt); free(hvi); return -1; }
    uint8_t *hv_ok = (uint8_t *)malloc((size_t)N);
    double *hv = (double *)malloc(sizeof(double) * (size_t)N);
    int64_t *hv_ts = (int64_t *)malloc(sizeof(int64_t) * (size_t)N);
    for (int64_t n = 0; n < N; n++) { hv_ok[n] = 1; hv[n] = (double)hvi[n]; hv_ts[n] = now_ns; }
    usage_src src;
    memset(&src, 0, sizeof src);
    src.soa = 1; src.ok = ok; src.val = val; src.ts = ts; src.N = N;
    src.hv_ok = hv_ok; src.hv = hv; src.hv_ts = hv_ts;
    int32_t *pr = map_rows(pol->n_pred, pol->pred_name, K, key_names);
    int32_t *qr = map_rows(pol->n_prio, pol->prio_name, K, key_names);
    src.pred_row = pr; src.prio_row = qr;
    /* per-node state: feasible flag and score under the current hot value */
    int8_t *feas = (int8_t *)malloc((size_t)N);
    int64_t *sc = (int64_t *)malloc(sizeof(int64_t) * (size_t)N);
    for (int64_t n = 0; n < N; n++) {
        feas[n] = filter_one(pol, &src, n, now_ns, 0) < 0;
        sc[n] = score_one(pol, &src, n, now_ns);
    }
    for (int64_t p = 0; p < P; p++) {
        int ds = pod_ds ? pod_ds[p] : 0;
        int64_t best = -1, bs = -1;
        for (int64_t n = 0; n < N; n++)
            if ((ds || feas[n]) && sc[n] > bs) { bs = sc[n]; best = n; }
        chosen[p] = best;
        if (best < 0) continue;
        /* new Binding{Timestamp: now_unix} on node `best` */
        int64_t v = 0;
        for (int32_t w = 0; w < W; w++) {
            int64_t timeline = now_unix - or_go_duration_seconds_trunc(pol->hot_tr_ns[w]);
            if (now_unix > timeline) cnt[(size_t)w * (size_t)N + (size_t)best]++;
            v += cnt[(size_t)w * (size_t)N + (size_t)best] / pol->hot_count[w];
        }
        hv[best] = (double)v;
        sc[best] = score_one(pol, &src, best, now_ns);
    }
    free(cnt); free(hvi); free(hv_ok); free(hv); free(hv_ts); free(pr); free(qr); free(feas); free(sc);
    return 0;
}

/* ------------------------------------------------------------------ */
/* BindingRecords (pkg/controller/annotator/binding.go:50-123) over go1.17
 * container/heap (src/container/heap/heap.go): Push = append + up(n-1),
 * Pop = Swap(0, n-1) + down(0, n-1) + remove last; Less = Timestamp <.
 * ops[i] = 0: AddBinding{node[i], Timestamp arg[i]} (pops the minimum first
 * when Len() == size, binding.go:69-78); ops[i] = 1: BindingsGC at
 * time.Now().UTC().Unix() = arg[i] (binding.go:100-123).  The final heap array
 * (Go's slice order) goes to out_node/out_ts, its length to *out_len.
 * Returns -1 for size <= 0 (AddBinding on a 0-size heap pops an empty heap).  */
typedef struct {
    int32_t node;
    int64_t ts;
} or_binding;

static void bh_swap(or_binding *h, int64_t i, int64_t j) {
    or_binding t = h[i];
    h[i] = h[j];
    h[j] = t;
}
static void bh_up(or_binding *h, int64_t j) {
    for (;;) {
        int64_t i = (j - 1) / 2; /* parent; Go truncates (-1)/2 to 0 */
        if (i == j || !(h[j].ts < h[i].ts)) break;
        bh_swap(h, i, j);
        j = i;
    }
}
static void bh_down(or_binding *h, int64_t i0, int64_t n) {
    int64_t i = i0;
    for (;;) {
        int64_t j1 = 2 * i + 1;
        if (j1 >= n || j1 < 0) break;
        int64_t j = j1;
        int64_t j2 = j1 + 1;
        if (j2 < n && h[j2].ts < h[j1].ts) j = j2;
        if (!(h[j].ts < h[i].ts)) break;
        bh_swap(h, i, j);
        i = j;
    }
}
static or_binding bh_pop(or_binding *h, int64_t *len) {
    int64_t n = *len - 1;
    bh_swap(h, 0, n);
    bh_down(h, 0, n);
    *len = n;
    return h[n];
}
static void bh_push(or_binding *h, int64_t *len, or_binding b) {
    h[*len] = b;
    (*len)++;
    bh_up(h, *len - 1);
}

int or_binding_heap(int64_t size, int64_t gc_tr_ns, int64_t n_ops, const uint8_t *ops, const int32_t *node,
                    const int64_t *arg, int64_t *out_len, int32_t *out_node, int64_t *out_ts) {
    if (size <= 0) return -1;
    or_binding *h = (or_binding *)malloc(sizeof(or_binding) * (size_t)(size + 1));
    if (!h) return -2;
    int64_t len = 0;
    for (int64_t i = 0; i < n_ops; ++i) {
        if (ops[i] == 0) {
            if (len == size) (void)bh_pop(h, &len);
            or_binding b = {node[i], arg[i]};
            bh_push(h, &len, b);
        } else {
            if (gc_tr_ns == 0) continue;
            int64_t timeline = arg[i] - or_go_duration_seconds_trunc(gc_tr_ns);
            while (len > 0) {
                or_binding b = bh_pop(h, &len);
                if (b.ts > timeline) {
                    bh_push(h, &len, b);
                    break;
                }
            }
        }
    }
    *out_len = len;
    for (int64_t i = 0; i < len; ++i) {
        out_node[i] = h[i].node;
        out_ts[i] = h[i].ts;
    }
    free(h);
    return 0;
}
