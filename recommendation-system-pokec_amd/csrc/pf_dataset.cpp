// pf_dataset.cpp — the reference's start-up loaders (include/pokec_io.h), restated
// for the product: api_cli.cpp:86-167 reads text columns, adjacency, encoded users,
// the median age and the normalisers, then hands the maps to Recommender.  Here the
// result is a pf_corpus_desc for pf_open plus the reference's own hash containers
// (same key types, same insertion sequence), which fix every iteration order the
// reference exposes: the profiles map (hold-out drivers), adj_list, and each
// token_cols map (profile JSON).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "pf_batch.h"
#include "pf_debug.h"
#include "pokec_io.h"

namespace pf {
void set_open_error(const std::string& m);
}

namespace {

constexpr int kFixed = PF_NUM_FIXED;
const char* const kFixedKeys[kFixed] = {"public", "gender", "completion", "age", "region", "clubs", "friends"};

// split_csv_line (utils.cpp:36-50): '"' toggles quoting and is dropped, no escapes.
// Reuses the strings of `out` (assign keeps their capacity).
void split_csv(const std::string& line, std::vector<std::string>& out, size_t& n) {
    n = 0;
    auto next = [&]() -> std::string& {
        if (n == out.size()) out.emplace_back();
        std::string& s = out[n++];
        s.clear();
        return s;
    };
    std::string* cur = &next();
    bool q = false;
    for (char c : line) {
        if (c == '"') { q = !q; continue; }
        if (c == ',' && !q) cur = &next();
        else cur->push_back(c);
    }
}

// split_csv_line_local (vocab_builder.cpp:123-131): as above, plus "" inside quotes = '"'
std::vector<std::string> split_csv_local(const std::string& line) {
    std::vector<std::string> out;
    std::string cur;
    bool q = false;
    for (size_t i = 0; i < line.size(); ++i) {
        const char c = line[i];
        if (c == '"') {
            if (q && i + 1 < line.size() && line[i + 1] == '"') { cur.push_back('"'); ++i; continue; }
            q = !q;
            continue;
        }
        if (c == ',' && !q) { out.push_back(cur); cur.clear(); }
        else cur.push_back(c);
    }
    out.push_back(cur);
    return out;
}

// std::getline(stringstream(s), tok, sep) tokens: [b, e) ranges of s; no trailing empty token
template <class F>
void for_each_token(const std::string& s, char sep, F&& f) {
    size_t b = 0;
    const size_t n = s.size();
    while (b < n) {
        size_t e = s.find(sep, b);
        if (e == std::string::npos) e = n;
        f(b, e);
        b = e + 1;
    }
}

// C atoi of s[b..): stops at the first non-digit, which the separators (';' ':' ',') are
int atoi_at(const std::string& s, size_t b) { return atoi(s.c_str() + b); }

bool is_space(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

// One parsed users_encoded row (UserProfile, include/user_profile.h:10-20)
struct Row {
    int32_t uid, pub, comp, gen, age;
    int32_t reg[3];
    std::vector<uint32_t> clubs, friends;
    std::vector<int32_t> col_off;                 // T+1 offsets into tok
    std::vector<std::pair<int32_t, int32_t>> tok; // per column: first-insertion order, last value
};

}  // namespace

struct pf_dataset {
    // a carried pf_eval_recommendation_tests_async call reads rows / profiles when its last chunk is
    // unpacked: it holds the dataset (DsHold), and pf_dataset_free of a held dataset defers the delete
    // to the last holder
    std::mutex hold_mu;
    int holds = 0;
    bool free_pending = false;
    std::vector<std::string> cols;
    std::vector<Row> rows;                             // slot = first appearance of the uid
    std::unordered_map<int, int32_t> profiles;         // uid -> slot, built like out_profiles
    std::unordered_map<int, std::vector<int>> adj_list;// built like build_adj_list(gb.adjacency)
    std::vector<int32_t> adj_seq;                      // adj_list's key insertion sequence (binary cache)
    std::unordered_map<std::string, std::pair<float, float>> norms;
    std::unordered_map<int, std::string> club_names;
    pf_dataset_info info{};
    // pf_corpus_desc storage
    std::vector<int32_t> uid, pub, comp, gen, age, reg, tok_tid, tok_tf, adj_uid, adj_nbr;
    std::vector<int64_t> club_off, friend_off, tok_off, adj_off;
    std::vector<uint32_t> club_ids, friend_ids;
    std::vector<uint8_t> npres;
    std::vector<float> nmean, nsd;
    pf_corpus_desc desc{};
    // the hold-out drivers' sampled plans: a pure function of the loaded maps and the sample
    // size (test.cpp:13-60, recommendation_tests.cpp:68-100 sampling), so built once per
    // (driver, size) and shared by every later call and engine context
    mutable std::mutex plan_mu;
    mutable std::unordered_map<int64_t, std::shared_ptr<const void>> plans;
};

namespace {

int fail(const std::string& m) {
    pf::set_open_error(m);
    return PF_EINVAL;
}

// load_text_columns_from_file (utils.cpp:13-24)
bool load_columns(const std::string& path, std::vector<std::string>& out) {
    std::ifstream in(path);
    if (!in.is_open()) return false;
    std::string line;
    while (std::getline(in, line))
        if (!line.empty()) out.push_back(line);
    return true;
}

// ---------------------------------------------------------------- parallel text ingest (F2)
// The reference reads both CSVs line by line with std::getline (graph_builder.cpp:44,
// user_loader.cpp:38).  Here the file is read whole, cut into the same lines ('\n' only; a
// '\r' stays in the line, a last line without '\n' still counts), the lines are parsed on
// threads, and the parsed records are inserted into the hash containers on one thread in
// file order, so every container sees the reference's insertion sequence.

bool read_file(const std::string& path, std::string& buf) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    buf.clear();
    char tmp[1 << 16];
    if (fseek(f, 0, SEEK_END) == 0) {
        const long sz = ftell(f);
        if (sz > 0) buf.reserve((size_t)sz);
        fseek(f, 0, SEEK_SET);
    }
    size_t got;
    while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, got);
    const bool ok = !ferror(f);
    fclose(f);
    return ok;
}

// [begin, end) of each std::getline line of buf from offset `from`, at most max_lines (<= 0: all)
void split_lines(const std::string& buf, size_t from, int64_t max_lines, std::vector<std::pair<size_t, size_t>>& out) {
    out.clear();
    const char* p = buf.data();
    const size_t n = buf.size();
    size_t b = from;
    while (b < n && (max_lines <= 0 || (int64_t)out.size() < max_lines)) {
        const void* q = memchr(p + b, '\n', n - b);
        const size_t e = q ? (size_t)((const char*)q - p) : n;
        out.emplace_back(b, e);
        b = e + 1;
    }
}

int ingest_threads() {
    const long v = pf::debug_long("load_threads", 0);  // PF_DEBUG load_threads (tests, tools)
    if (v > 0) return (int)std::min<long>(v, 256);
    const unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
}

// f(i) for i in [0, n) on ingest_threads() threads, contiguous chunks of `grain`
template <class F>
void parallel_for(size_t n, size_t grain, F f) {
    const int nt = (int)std::min<size_t>((size_t)ingest_threads(), (n + grain - 1) / std::max<size_t>(grain, 1));
    if (nt <= 1) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (;;) {
            const size_t b = next.fetch_add(grain);
            if (b >= n) return;
            const size_t e = std::min(n, b + grain);
            for (size_t i = b; i < e; ++i) f(i);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
}

// GraphBuilder::load_serialized (graph_builder.cpp:39-59) + build_adj_list (utils.cpp:26-34)
bool load_adjacency(const std::string& path, std::unordered_map<int, std::vector<int>>& adj_list,
                    std::vector<int32_t>& adj_seq) {
    std::string buf;
    if (!read_file(path, buf)) return false;
    std::vector<std::pair<size_t, size_t>> lines;
    split_lines(buf, 0, 0, lines);
    // one line "uid,n1,n2,..." -> (uid, neighbours); tokens trimmed (trim_copy_g), empty skipped
    std::vector<int> uid(lines.size(), -1);
    std::vector<std::vector<int>> nb(lines.size());
    parallel_for(lines.size(), 4096, [&](size_t i) {
        const size_t lb = lines[i].first, le = lines[i].second;
        bool first = true;
        size_t b = lb;
        while (b < le) {
            const void* q = memchr(buf.data() + b, ',', le - b);
            const size_t e = q ? (size_t)((const char*)q - buf.data()) : le;
            size_t s = b;
            while (s < e && is_space((unsigned char)buf[s])) ++s;
            if (s < e) {
                const int v = atoi(buf.c_str() + s);  // stops at ',' like atoi on the token copy
                if (first) { uid[i] = v; first = false; }
                else nb[i].push_back(v);
            }
            b = e + 1;
        }
    });
    std::unordered_map<int, std::vector<int>> adjacency;  // GraphBuilder::adjacency
    for (size_t i = 0; i < lines.size(); ++i) {
        if (nb[i].empty()) continue;  // adjacency[uid] is touched only by a push_back
        std::vector<int>& a = adjacency[uid[i]];
        if (a.empty()) a = std::move(nb[i]);  // a repeated uid line appends
        else a.insert(a.end(), nb[i].begin(), nb[i].end());
    }
    adj_seq.clear();
    adj_seq.reserve(adjacency.size());
    for (auto& kv : adjacency) {  // build_adj_list: out[u].push_back in adjacency order
        adj_seq.push_back(kv.first);
        std::vector<int>& o = adj_list[kv.first];
        if (o.empty()) o = std::move(kv.second);
        else o.insert(o.end(), kv.second.begin(), kv.second.end());
    }
    return true;
}

// One users_encoded data line -> r (user_loader.cpp:40-88); false for an empty line or uid 0
bool parse_user(const std::string& line, size_t T, std::vector<std::string>& parts, Row& r) {
    if (line.empty()) return false;
    size_t np = 0;
    split_csv(line, parts, np);
    const int uid = atoi(parts[0].c_str());
    if (uid == 0) return false;
    auto has = [&](size_t i) { return i < np && !parts[i].empty(); };
    r.uid = uid;
    r.pub = has(1) ? atoi(parts[1].c_str()) : -1;
    r.comp = has(2) ? atoi(parts[2].c_str()) : -1;
    r.gen = has(3) ? atoi(parts[3].c_str()) : -1;
    r.age = has(5) ? atoi(parts[5].c_str()) : 0;
    if (has(6))
        for_each_token(parts[6], ';', [&](size_t b, size_t e) {
            if (b < e) r.clubs.push_back((uint32_t)atoi_at(parts[6], b));
        });
    if (has(7))
        for_each_token(parts[7], ';', [&](size_t b, size_t e) {
            if (b < e) r.friends.push_back((uint32_t)atoi_at(parts[7], b));
        });
    r.reg[0] = r.reg[1] = r.reg[2] = -1;
    if (has(4)) {
        std::string rf = parts[4];
        if (rf.size() >= 2 && rf.front() == '"' && rf.back() == '"') rf = rf.substr(1, rf.size() - 2);
        int pi = 0;
        for_each_token(rf, ';', [&](size_t b, size_t e) {
            if (pi >= 3) return;
            if (b < e) r.reg[pi] = atoi_at(rf, b);
            ++pi;
        });
    }
    r.col_off.resize(T + 1);
    for (size_t t = 0; t < T; ++t) {
        r.col_off[t] = (int32_t)r.tok.size();
        const size_t idx = 8 + t;
        if (!has(idx)) continue;
        std::string s = parts[idx];  // parse_tok_field (utils.cpp:52-68)
        if (s.size() >= 2 && s.front() == '"' && s.back() == '"') s = s.substr(1, s.size() - 2);
        const size_t base = r.tok.size();
        for_each_token(s, ';', [&](size_t b, size_t e) {
            if (b == e) return;
            const size_t p = s.find(':', b);
            if (p == std::string::npos || p >= e) return;
            const int tid = atoi_at(s, b), cnt = atoi_at(s, p + 1);
            // token_cols[t][tid] = cnt: a repeated tid keeps its first position, takes the last count
            for (size_t k = base; k < r.tok.size(); ++k)
                if (r.tok[k].first == tid) { r.tok[k].second = cnt; return; }
            r.tok.emplace_back(tid, cnt);
        });
    }
    r.col_off[T] = (int32_t)r.tok.size();
    return true;
}

// load_users_encoded (user_loader.cpp:10-96)
bool load_users(const std::string& path, int64_t max_lines, pf_dataset& d) {
    std::string buf;
    if (!read_file(path, buf)) return false;
    const void* h = memchr(buf.data(), '\n', buf.size());
    if (buf.empty()) return false;  // no header line
    const size_t from = h ? (size_t)((const char*)h - buf.data()) + 1 : buf.size();
    std::vector<std::pair<size_t, size_t>> lines;
    split_lines(buf, from, max_lines, lines);
    const size_t T = d.cols.size();
    std::vector<Row> parsed(lines.size());
    std::vector<uint8_t> ok(lines.size(), 0);
    const size_t grain = 2048;
    parallel_for((lines.size() + grain - 1) / grain, 1, [&](size_t g) {
        std::vector<std::string> parts;
        std::string line;
        const size_t e = std::min(lines.size(), (g + 1) * grain);
        for (size_t i = g * grain; i < e; ++i) {
            line.assign(buf, lines[i].first, lines[i].second - lines[i].first);
            ok[i] = parse_user(line, T, parts, parsed[i]) ? 1 : 0;
        }
    });
    std::string().swap(buf);
    d.rows.reserve(lines.size());  // (the profiles map is not reserved: its bucket sequence, and
                                   // so its iteration order, stays the reference's)
    for (size_t i = 0; i < lines.size(); ++i) {
        if (!ok[i]) continue;
        // out_profiles[p.user_id] = std::move(p): a repeated uid replaces the profile in place
        auto ins = d.profiles.emplace(parsed[i].uid, (int32_t)d.rows.size());
        if (ins.second) d.rows.push_back(std::move(parsed[i]));
        else d.rows[ins.first->second] = std::move(parsed[i]);
    }
    d.info.lines_read = (int64_t)lines.size();
    return true;
}

// load_column_normalizers (utils.cpp:123-142)
bool load_norms(const std::string& path, std::unordered_map<std::string, std::pair<float, float>>& out) {
    std::ifstream in(path);
    if (!in.is_open()) return false;
    std::string line;
    if (!std::getline(in, line)) return false;
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        const size_t p1 = line.find(',');
        if (p1 == std::string::npos) continue;
        const size_t p2 = line.find(',', p1 + 1);
        const std::string col = line.substr(0, p1);
        if (p2 == std::string::npos) continue;
        const float mean = (float)atof(line.substr(p1 + 1, p2 - (p1 + 1)).c_str());
        const float sd = (float)atof(line.substr(p2 + 1).c_str());
        out[col] = std::make_pair(mean, sd);
    }
    return !out.empty();
}

// VocabBuilder::load_vocab (vocab_builder.cpp:133-197): only the club map is used by the
// path (api_cli.cpp:169-170); tokens.csv must exist and have a header for it to load.
bool load_club_names(const std::string& dir, std::unordered_map<int, std::string>& names) {
    {
        std::ifstream tok(dir + "/tokens.csv");
        std::string header;
        if (!tok.is_open() || !std::getline(tok, header)) return false;
    }
    std::unordered_map<std::string, int> club_to_id;
    std::ifstream in(dir + "/clubs_map.csv");
    if (in.is_open()) {
        std::string line;
        if (std::getline(in, line)) {
            while (std::getline(in, line)) {
                if (line.empty()) continue;
                std::vector<std::string> cols = split_csv_local(line);
                if (cols.size() < 3) continue;
                club_to_id[cols[1]] = atoi(cols[0].c_str());
            }
        }
    }
    for (auto& kv : club_to_id) names[kv.second] = kv.first;  // api_cli.cpp:169-170
    return true;
}

void build_desc(pf_dataset& d) {
    const int32_t n = (int32_t)d.rows.size(), T = (int32_t)d.cols.size();
    d.uid.resize(n); d.pub.resize(n); d.comp.resize(n); d.gen.resize(n); d.age.resize(n);
    d.reg.resize((size_t)3 * n);
    // row i's lists go to offsets fixed by a prefix pass, then rows are copied on threads
    d.club_off.assign((size_t)n + 1, 0); d.friend_off.assign((size_t)n + 1, 0);
    d.tok_off.assign((size_t)n * T + 1, 0);
    std::vector<int64_t> tbase((size_t)n + 1, 0);
    for (int32_t i = 0; i < n; ++i) {
        const Row& r = d.rows[i];
        d.club_off[i + 1] = d.club_off[i] + (int64_t)r.clubs.size();
        d.friend_off[i + 1] = d.friend_off[i] + (int64_t)r.friends.size();
        tbase[i + 1] = tbase[i] + (int64_t)r.tok.size();
    }
    d.club_ids.resize((size_t)d.club_off[n]); d.friend_ids.resize((size_t)d.friend_off[n]);
    d.tok_tid.resize((size_t)tbase[n]); d.tok_tf.resize((size_t)tbase[n]);
    parallel_for((size_t)n, 8192, [&](size_t i) {
        const Row& r = d.rows[i];
        d.uid[i] = r.uid; d.pub[i] = r.pub; d.comp[i] = r.comp; d.gen[i] = r.gen; d.age[i] = r.age;
        for (int k = 0; k < 3; ++k) d.reg[(size_t)3 * i + k] = r.reg[k];
        std::copy(r.clubs.begin(), r.clubs.end(), d.club_ids.begin() + d.club_off[i]);
        std::copy(r.friends.begin(), r.friends.end(), d.friend_ids.begin() + d.friend_off[i]);
        const int64_t tb = tbase[i];
        for (size_t k = 0; k < r.tok.size(); ++k) {
            d.tok_tid[(size_t)tb + k] = r.tok[k].first;
            d.tok_tf[(size_t)tb + k] = r.tok[k].second;
        }
        for (int32_t t = 0; t < T; ++t) d.tok_off[(size_t)i * T + t + 1] = tb + r.col_off[t + 1];
    });
    // adjacency rows in adj_list's iteration order
    std::vector<const std::vector<int>*> arow;
    arow.reserve(d.adj_list.size());
    d.adj_uid.clear();
    d.adj_uid.reserve(d.adj_list.size());
    d.adj_off.assign(1, 0);
    d.adj_off.reserve(d.adj_list.size() + 1);
    for (auto& kv : d.adj_list) {
        d.adj_uid.push_back(kv.first);
        arow.push_back(&kv.second);
        d.adj_off.push_back(d.adj_off.back() + (int64_t)kv.second.size());
    }
    d.adj_nbr.resize((size_t)d.adj_off.back());
    parallel_for(arow.size(), 8192, [&](size_t j) {
        std::copy(arow[j]->begin(), arow[j]->end(), d.adj_nbr.begin() + d.adj_off[j]);
    });
    // one map feeds both normaliser sets (api_cli.cpp:163-165)
    const int K = kFixed + T;
    d.npres.assign(K, 0); d.nmean.assign(K, 0.f); d.nsd.assign(K, 0.f);
    for (int k = 0; k < K; ++k) {
        auto it = d.norms.find(k < kFixed ? std::string(kFixedKeys[k]) : d.cols[k - kFixed]);
        if (it == d.norms.end()) continue;
        d.npres[k] = 1;
        d.nmean[k] = it->second.first;
        d.nsd[k] = it->second.second;
    }
    pf_corpus_desc& c = d.desc;
    c = pf_corpus_desc{};
    c.n_users = n;
    c.n_cols = T;
    c.user_id = d.uid.data(); c.public_flag = d.pub.data(); c.completion = d.comp.data();
    c.gender = d.gen.data(); c.age = d.age.data(); c.region = d.reg.data();
    c.club_off = d.club_off.data(); c.club_ids = d.club_ids.data();
    c.friend_off = d.friend_off.data(); c.friend_ids = d.friend_ids.data();
    c.tok_off = d.tok_off.data(); c.tok_tid = d.tok_tid.data(); c.tok_tf = d.tok_tf.data();
    c.n_adj = (int32_t)d.adj_uid.size();
    c.adj_uid = d.adj_uid.data(); c.adj_off = d.adj_off.data(); c.adj_nbr = d.adj_nbr.data();
    c.idf_mode = PF_IDF_FROM_PROFILES;  // rec.compute_idf_from_profiles(textCols), api_cli.cpp:162
    c.norm_present = d.npres.data(); c.norm_mean = d.nmean.data(); c.norm_sd = d.nsd.data();
}

// ---------------------------------------------------------------- binary cache (F2)
// The parse phase's output (the rows in slot order, the user loader's line count, the
// adjacency rows in adj_list's insertion sequence) as flat little-endian arrays, keyed by
// the two CSVs' sizes and mtimes, the line cap and the text columns.  Re-inserting the
// uids and adjacency keys in the recorded sequences rebuilds both hash containers with
// the reference's iteration orders; everything after the parse (median, normalisers,
// club names, corpus arrays) runs as without the cache.
constexpr char kCacheMagic[8] = {'P', 'F', 'D', 'S', 'C', 'A', 'C', '1'};

struct CacheKey {
    bool ok = false;
    int64_t max_lines = 0, u_size = 0, u_mtime = 0, a_size = 0, a_mtime = 0;
    std::string cols;  // names joined by '\n'
};

CacheKey cache_key(const std::string& data, int64_t max_lines, const std::vector<std::string>& cols) {
    CacheKey k;
    struct stat su, sa;
    if (stat((data + "/users_encoded.csv").c_str(), &su) != 0 || stat((data + "/adjacency.csv").c_str(), &sa) != 0)
        return k;
    k.max_lines = max_lines <= 0 ? 0 : max_lines;
    k.u_size = (int64_t)su.st_size;
    k.u_mtime = (int64_t)su.st_mtim.tv_sec * 1000000000LL + su.st_mtim.tv_nsec;
    k.a_size = (int64_t)sa.st_size;
    k.a_mtime = (int64_t)sa.st_mtim.tv_sec * 1000000000LL + sa.st_mtim.tv_nsec;
    for (auto& c : cols) { k.cols += c; k.cols += '\n'; }
    k.ok = true;
    return k;
}

// Arrays are written straight to the file as (int64 count, raw elements).
struct Writer {
    FILE* f;
    bool ok = true;
    void raw(const void* p, size_t n) { if (ok && n) ok = fwrite(p, 1, n, f) == n; }
    template <class T> void put(const T& v) { raw(&v, sizeof(T)); }
    template <class T> void arr(const std::vector<T>& v) {
        put((int64_t)v.size());
        raw(v.data(), sizeof(T) * v.size());
    }
};

// The cache file mapped read-only; arrays are used in place.
struct Reader {
    const char* p;
    const char* e;
    bool ok = true;
    template <class T> T get() {
        T v{};
        if ((size_t)(e - p) < sizeof(T)) { ok = false; return v; }
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    template <class T> const T* arr(size_t& n) {  // elements are 4- or 8-byte aligned (see write_cache)
        const int64_t k = get<int64_t>();
        if (!ok || k < 0 || (uint64_t)k > (uint64_t)(e - p) / sizeof(T)) { ok = false; n = 0; return nullptr; }
        const T* v = reinterpret_cast<const T*>(p);
        n = (size_t)k;
        p += sizeof(T) * n;
        return v;
    }
};

std::string key_bytes(const CacheKey& k) {
    std::string b(kCacheMagic, 8);
    auto put = [&](int64_t v) { b.append(reinterpret_cast<const char*>(&v), 8); };
    put(k.max_lines); put(k.u_size); put(k.u_mtime); put(k.a_size); put(k.a_mtime);
    put((int64_t)k.cols.size());
    b += k.cols;
    b.append((8 - b.size() % 8) % 8, '\0');  // keep the arrays 8-byte aligned
    return b;
}

void write_cache(const std::string& path, const CacheKey& key, const pf_dataset& d) {
    const size_t n = d.rows.size(), T = d.cols.size();
    std::vector<int32_t> fixed(n * 8);
    std::vector<int64_t> coff(n + 1, 0), foff(n + 1, 0), toff(n + 1, 0);
    std::vector<uint16_t> cnt(n * T + (4 - (n * T) % 4) % 4);  // padded to 8 bytes
    for (size_t i = 0; i < n; ++i) {
        const Row& r = d.rows[i];
        int32_t* f = &fixed[i * 8];
        f[0] = r.uid; f[1] = r.pub; f[2] = r.comp; f[3] = r.gen; f[4] = r.age;
        f[5] = r.reg[0]; f[6] = r.reg[1]; f[7] = r.reg[2];
        coff[i + 1] = coff[i] + (int64_t)r.clubs.size();
        foff[i + 1] = foff[i] + (int64_t)r.friends.size();
        toff[i + 1] = toff[i] + (int64_t)r.tok.size();
        for (size_t t = 0; t < T; ++t) {
            const int32_t k = r.col_off[t + 1] - r.col_off[t];
            if (k > 65535) return;  // not cacheable (16-bit per-column counts)
            cnt[i * T + t] = (uint16_t)k;
        }
    }
    std::vector<uint32_t> clubs((size_t)coff[n] + (coff[n] & 1)), friends((size_t)foff[n] + (foff[n] & 1));
    std::vector<std::pair<int32_t, int32_t>> tok((size_t)toff[n]);
    parallel_for(n, 8192, [&](size_t i) {
        const Row& r = d.rows[i];
        std::copy(r.clubs.begin(), r.clubs.end(), clubs.begin() + coff[i]);
        std::copy(r.friends.begin(), r.friends.end(), friends.begin() + foff[i]);
        std::copy(r.tok.begin(), r.tok.end(), tok.begin() + toff[i]);
    });
    std::vector<int64_t> aoff(1, 0);
    std::vector<int32_t> aseq(d.adj_seq), anbr;
    for (int32_t u : d.adj_seq) {
        const std::vector<int>& v = d.adj_list.at(u);
        anbr.insert(anbr.end(), v.begin(), v.end());
        aoff.push_back((int64_t)anbr.size());
    }
    if (aseq.size() & 1) aseq.push_back(0);  // padding (the real count is aoff.size() - 1)
    if (anbr.size() & 1) anbr.push_back(0);
    const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
    Writer w{fopen(tmp.c_str(), "wb")};
    if (!w.f) return;
    const std::string kb = key_bytes(key);
    w.raw(kb.data(), kb.size());
    w.put(d.info.lines_read);
    w.put((int64_t)n);
    w.put((int64_t)coff[n]); w.put((int64_t)foff[n]); w.put((int64_t)aoff.back());
    w.arr(fixed); w.arr(coff); w.arr(clubs); w.arr(foff); w.arr(friends); w.arr(toff); w.arr(cnt); w.arr(tok);
    w.arr(aseq); w.arr(aoff); w.arr(anbr);
    const bool ok = w.ok;
    if (fclose(w.f) != 0 || !ok || rename(tmp.c_str(), path.c_str()) != 0) remove(tmp.c_str());
}

bool read_cache(const std::string& path, const CacheKey& key, pf_dataset& d) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size <= 0) { close(fd); return false; }
    const size_t len = (size_t)st.st_size;
    void* m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return false;
    struct Unmap { void* m; size_t len; ~Unmap() { munmap(m, len); } } unmap{m, len};
    const char* base = static_cast<const char*>(m);
    const std::string kb = key_bytes(key);
    if (len < kb.size() || std::memcmp(base, kb.data(), kb.size()) != 0) return false;  // stale or foreign
    Reader rd{base + kb.size(), base + len};
    const size_t T = d.cols.size();
    const int64_t lines = rd.get<int64_t>();
    const size_t n = (size_t)rd.get<int64_t>();
    const int64_t nclub = rd.get<int64_t>(), nfr = rd.get<int64_t>(), nadj = rd.get<int64_t>();
    size_t nfixed, ncoff, nclubs, nfoff, nfriends, ntoff, ncnt, ntok, naseq, naoff, nanbr;
    const int32_t* fixed = rd.arr<int32_t>(nfixed);
    const int64_t* coff = rd.arr<int64_t>(ncoff);
    const uint32_t* clubs = rd.arr<uint32_t>(nclubs);
    const int64_t* foff = rd.arr<int64_t>(nfoff);
    const uint32_t* friends = rd.arr<uint32_t>(nfriends);
    const int64_t* toff = rd.arr<int64_t>(ntoff);
    const uint16_t* cnt = rd.arr<uint16_t>(ncnt);
    const std::pair<int32_t, int32_t>* tok = rd.arr<std::pair<int32_t, int32_t>>(ntok);
    const int32_t* aseq = rd.arr<int32_t>(naseq);
    const int64_t* aoff = rd.arr<int64_t>(naoff);
    const int32_t* anbr = rd.arr<int32_t>(nanbr);
    if (!rd.ok || rd.p != rd.e || nfixed != n * 8 || ncoff != n + 1 || nfoff != n + 1 || ntoff != n + 1 ||
        ncnt < n * T || coff[n] != nclub || foff[n] != nfr || nclubs < (size_t)nclub || nfriends < (size_t)nfr ||
        toff[n] != (int64_t)ntok || naoff < 1 || naseq < naoff - 1 || aoff[naoff - 1] != nadj || nanbr < (size_t)nadj)
        return false;
    for (size_t i = 0; i < n; ++i)  // offsets must be monotone before rows index through them
        if (coff[i + 1] < coff[i] || foff[i + 1] < foff[i] || toff[i + 1] < toff[i]) return false;
    for (size_t j = 0; j + 1 < naoff; ++j)
        if (aoff[j + 1] < aoff[j]) return false;
    d.rows.clear();
    d.rows.resize(n);
    std::atomic<bool> bad{false};
    parallel_for(n, 8192, [&](size_t i) {
        Row& r = d.rows[i];
        const int32_t* f = &fixed[i * 8];
        r.uid = f[0]; r.pub = f[1]; r.comp = f[2]; r.gen = f[3]; r.age = f[4];
        r.reg[0] = f[5]; r.reg[1] = f[6]; r.reg[2] = f[7];
        r.clubs.assign(clubs + coff[i], clubs + coff[i + 1]);
        r.friends.assign(friends + foff[i], friends + foff[i + 1]);
        r.tok.assign(tok + toff[i], tok + toff[i + 1]);
        r.col_off.resize(T + 1);
        r.col_off[0] = 0;
        for (size_t t = 0; t < T; ++t) r.col_off[t + 1] = r.col_off[t] + cnt[i * T + t];
        if ((int64_t)r.col_off[T] != toff[i + 1] - toff[i]) bad = true;
    });
    if (bad) { d.rows.clear(); return false; }
    for (size_t i = 0; i < n; ++i) d.profiles.emplace(d.rows[i].uid, (int32_t)i);  // slot order = first appearance
    d.adj_seq.assign(aseq, aseq + (naoff - 1));
    for (size_t j = 0; j + 1 < naoff; ++j) d.adj_list[aseq[j]].assign(anbr + aoff[j], anbr + aoff[j + 1]);
    d.info.lines_read = lines;
    return true;
}

void write_int_list(std::string& o, const std::vector<uint32_t>& v) {
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) o += ',';
        o += std::to_string(v[i]);
    }
}

}  // namespace

extern "C" {

int pf_dataset_load(const char* root, int64_t max_lines, pf_dataset** out) {
    return pf_dataset_load_cached(root, max_lines, nullptr, nullptr, out);
}

int pf_dataset_load_cached(const char* root, int64_t max_lines, const char* cache_path, int32_t* from_cache,
                           pf_dataset** out) {
    if (!root || !out) return fail("null argument");
    *out = nullptr;
    if (from_cache) *from_cache = 0;
    auto d = new pf_dataset();
    const std::string r(root), data = r + "/data";
    auto bail = [&](const std::string& m) { delete d; return fail(m); };
    if (!load_columns(r + "/config/text_columns.txt", d->cols)) return bail("cannot read config/text_columns.txt");
    if (d->cols.size() > PF_MAX_COLS) return bail("more than PF_MAX_COLS text columns");
    const bool prof = pf::debug_long("host_prof", 0) > 0;
    auto t0 = std::chrono::steady_clock::now();
    auto stage = [&](const char* what) {  // PF_DEBUG host_prof=1: loader stage clocks on stderr
        const auto t1 = std::chrono::steady_clock::now();
        if (prof) fprintf(stderr, "[pf_dataset_load] %s %.3f s\n", what, std::chrono::duration<double>(t1 - t0).count());
        t0 = t1;
    };
    const CacheKey key = cache_key(data, max_lines, d->cols);
    if (cache_path && key.ok && read_cache(cache_path, key, *d)) {
        if (from_cache) *from_cache = 1;
        stage("binary cache");
    } else {
        if (!load_adjacency(data + "/adjacency.csv", d->adj_list, d->adj_seq)) return bail("cannot read data/adjacency.csv");
        stage("adjacency");
        if (!load_users(data + "/users_encoded.csv", max_lines, *d)) return bail("cannot load users_encoded.csv");
        stage("users");
        if (cache_path && key.ok) {
            write_cache(cache_path, key, *d);  // best effort: a failed write leaves no file behind
            stage("cache write");
        }
    }
    // median age (api_cli.cpp:139-153, user_loader.cpp:98-140)
    int median = 0;
    bool loaded = false;
    {
        std::ifstream in(data + "/median_age.txt");
        std::string s;
        if (in.is_open() && std::getline(in, s)) { median = atoi(s.c_str()); loaded = true; }
    }
    if (!loaded) {
        std::vector<int> ages;
        for (const Row& row : d->rows)
            if (row.age > 0) ages.push_back(row.age);
        if (!ages.empty()) {
            std::sort(ages.begin(), ages.end());
            const size_t n = ages.size();
            median = n % 2 ? ages[n / 2] : (ages[n / 2 - 1] + ages[n / 2]) / 2;
        }
    }
    int replaced = 0;
    for (Row& row : d->rows)
        if (row.age == 0) { row.age = median; ++replaced; }
    load_norms(data + "/column_normalizers.csv", d->norms);
    d->info.vocab_loaded = load_club_names(data, d->club_names) ? 1 : 0;
    build_desc(*d);
    stage("ages, normalisers, club names, corpus arrays");
    d->info.n_profiles = (int32_t)d->rows.size();
    d->info.n_cols = (int32_t)d->cols.size();
    d->info.n_adj = (int32_t)d->adj_list.size();
    d->info.median_age = median;
    d->info.median_loaded = loaded ? 1 : 0;
    d->info.ages_replaced = replaced;
    d->info.n_normalizers = (int32_t)d->norms.size();
    d->info.n_club_names = (int32_t)d->club_names.size();
    *out = d;
    return PF_OK;
}

void pf_dataset_free(pf_dataset* ds) {
    if (!ds) return;
    {
        std::lock_guard<std::mutex> g(ds->hold_mu);
        if (ds->holds > 0) {  // a carried call still reads it: its last holder deletes it
            ds->free_pending = true;
            return;
        }
    }
    delete ds;
}

const pf_corpus_desc* pf_dataset_desc(const pf_dataset* ds) { return ds ? &ds->desc : nullptr; }

int pf_dataset_info_get(const pf_dataset* ds, pf_dataset_info* out) {
    if (!ds || !out) return PF_EINVAL;
    *out = ds->info;
    return PF_OK;
}

const char* pf_dataset_column(const pf_dataset* ds, int32_t t) {
    if (!ds || t < 0 || t >= (int32_t)ds->cols.size()) return nullptr;
    return ds->cols[t].c_str();
}

int pf_dataset_profile_order(const pf_dataset* ds, int32_t* out, int32_t cap, int32_t* n) {
    if (!ds || !n || (cap > 0 && !out)) return PF_EINVAL;
    int32_t i = 0;
    for (auto& kv : ds->profiles) {
        if (i < cap) out[i] = kv.first;
        ++i;
    }
    *n = i;
    return PF_OK;
}

int pf_dataset_adj_order(const pf_dataset* ds, int32_t* out, int32_t cap, int32_t* n) {
    if (!ds || !n || (cap > 0 && !out)) return PF_EINVAL;
    int32_t i = 0;
    for (auto& kv : ds->adj_list) {
        if (i < cap) out[i] = kv.first;
        ++i;
    }
    *n = i;
    return PF_OK;
}

// write_profile_json (api_cli.cpp:49-84)
int pf_dataset_profile_json(const pf_dataset* ds, int32_t uid, char* buf, int64_t cap, int64_t* len) {
    if (!ds || !len || (cap > 0 && !buf)) return PF_EINVAL;
    auto it = ds->profiles.find(uid);
    if (it == ds->profiles.end()) { *len = 0; return PF_ENOTFOUND; }
    const Row& p = ds->rows[it->second];
    std::string o;
    o.reserve(1024);
    o += "{\"user_id\":" + std::to_string(p.uid) + ",";
    o += "\"public_flag\":" + std::to_string(p.pub) + ",";
    o += "\"completion_percentage\":" + std::to_string(p.comp) + ",";
    o += "\"gender\":" + std::to_string(p.gen) + ",";
    o += "\"age\":" + std::to_string(p.age) + ",";
    o += "\"region_parts\":[" + std::to_string(p.reg[0]) + "," + std::to_string(p.reg[1]) + "," +
         std::to_string(p.reg[2]) + "],";
    o += "\"clubs\":[";
    write_int_list(o, p.clubs);
    o += "],\"friends\":[";
    write_int_list(o, p.friends);
    o += "],\"token_cols\":[";
    const size_t T = ds->cols.size();
    for (size_t t = 0; t < T; ++t) {
        if (t) o += ',';
        o += '{';
        // the reference iterates its unordered_map<int,int>: rebuild it with the same
        // insertion sequence (first occurrences in field order) to get the same order
        std::unordered_map<int, int> m;
        for (int32_t k = p.col_off[t]; k < p.col_off[t + 1]; ++k) m[p.tok[k].first] = p.tok[k].second;
        bool first = true;
        for (auto& pr : m) {
            if (!first) o += ',';
            first = false;
            o += "\"" + std::to_string(pr.first) + "\":" + std::to_string(pr.second);
        }
        o += '}';
    }
    o += "]}";
    *len = (int64_t)o.size();
    if (cap > 0) {
        const size_t k = std::min<size_t>(o.size(), (size_t)cap - 1);
        std::memcpy(buf, o.data(), k);
        buf[k] = 0;
    }
    return PF_OK;
}

const char* pf_dataset_club_name(const pf_dataset* ds, int32_t club_id) {
    if (!ds) return nullptr;
    auto it = ds->club_names.find(club_id);
    return it == ds->club_names.end() ? nullptr : it->second.c_str();
}

}  // extern "C"

// ---------------------------------------------------------------- normalisers (A18)
#include <cmath>
#include <random>
#include <unordered_set>

namespace {

// vec_set_similarity_local (utils.cpp:83-92): B's entries (with duplicates) found in set(A)
float set_sim(const std::vector<uint32_t>& A, const std::vector<uint32_t>& B) {
    if (A.empty() || B.empty()) return 0.0f;
    std::unordered_set<uint32_t> a(A.begin(), A.end());
    int inter = 0;
    for (uint32_t v : B) inter += a.count(v) != 0;
    const double den = std::sqrt((double)A.size()) * std::sqrt((double)B.size());
    if (den <= 0.0) return 0.0f;
    return (float)((double)inter / den);
}

// region_similarity_local (utils.cpp:94-103)
float region_sim(const int32_t* A, const int32_t* B) {
    int ac = 0, bc = 0, m = 0;
    for (int i = 0; i < 3; ++i) {
        ac += A[i] >= 0;
        bc += B[i] >= 0;
        m += A[i] >= 0 && B[i] >= 0 && A[i] == B[i];
    }
    if (ac == 0 || bc == 0) return 0.0f;
    return (float)((double)m / (std::sqrt((double)ac) * std::sqrt((double)bc)));
}

// cosine_counts_maps_local (utils.cpp:105-121) on one column's (tid, tf) lists.  All its
// sums are of integer products, exact in double, so the map iteration order is moot.
float count_cosine(const std::pair<int32_t, int32_t>* a, int na, const std::pair<int32_t, int32_t>* b, int nb) {
    if (na == 0 || nb == 0) return 0.0f;
    double sa = 0.0, sb = 0.0, dot = 0.0;
    for (int i = 0; i < na; ++i) sa += (double)a[i].second * a[i].second;
    for (int j = 0; j < nb; ++j) sb += (double)b[j].second * b[j].second;
    if (sa <= 0.0 || sb <= 0.0) return 0.0f;
    for (int i = 0; i < na; ++i)
        for (int j = 0; j < nb; ++j)
            if (a[i].first == b[j].first) dot += (double)a[i].second * b[j].second;
    const double norm = std::sqrt(sa) * std::sqrt(sb);
    if (norm <= 0.0) return 0.0f;
    return (float)(dot / norm);
}

std::pair<float, float> mean_sd(const std::vector<double>& v) {  // utils.cpp:212-226
    if (v.empty()) return {0.0f, 1.0f};
    double mu = 0.0;
    for (double x : v) mu += x;
    mu /= (double)v.size();
    double s = 0.0;
    if (v.size() > 1) {
        for (double x : v) {
            const double d = x - mu;
            s += d * d;
        }
        s = std::sqrt(s / (double)(v.size() - 1));
        if (s == 0.0) s = 1.0;
    } else {
        s = 1.0;
    }
    return {(float)mu, (float)s};
}

}  // namespace

extern "C" int pf_compute_normalizers(const pf_dataset* ds, int32_t sample_size, int32_t comps_per_user,
                                      const char* save_csv, float* out_mean, float* out_sd) {
    if (!ds || sample_size < 0 || comps_per_user < 0) return fail("bad argument");
    const size_t T = ds->cols.size();
    static const char* const keys[kFixed] = {"public", "gender", "completion", "age", "region", "clubs", "friends"};
    std::unordered_map<std::string, std::pair<float, float>> result;
    if (!ds->profiles.empty()) {
        std::vector<int> ids;  // the profiles map in its iteration order (utils.cpp:163-164)
        ids.reserve(ds->profiles.size());
        for (auto& kv : ds->profiles) ids.push_back(kv.first);
        std::mt19937 rng(12345);
        std::uniform_int_distribution<size_t> dist(0, ids.size() - 1);
        const size_t need = (size_t)sample_size * (size_t)comps_per_user;
        std::unordered_set<uint64_t> seen;
        std::vector<std::vector<double>> text(T);
        std::unordered_map<std::string, std::vector<double>> field;  // insertion order as utils.cpp:170-171
        for (auto k : keys) field[k] = std::vector<double>();
        std::vector<double>* fv[kFixed];
        for (int k = 0; k < kFixed; ++k) fv[k] = &field[keys[k]];
        size_t attempts = 0;
        while (seen.size() < need && attempts < need * 10) {
            ++attempts;
            const int a = ids[dist(rng)];
            const int b = ids[dist(rng)];
            if (a == b) continue;
            uint32_t x = (uint32_t)a, y = (uint32_t)b;  // pair_key_uint64 (utils.cpp:70-75)
            if (x > y) std::swap(x, y);
            if (!seen.insert(((uint64_t)x << 32) | y).second) continue;
            const Row& A = ds->rows[ds->profiles.find(a)->second];
            const Row& B = ds->rows[ds->profiles.find(b)->second];
            fv[0]->push_back(A.pub >= 0 && B.pub >= 0 && A.pub == B.pub ? 1.0 : 0.0);
            fv[1]->push_back(A.gen >= 0 && B.gen >= 0 && A.gen == B.gen ? 1.0 : 0.0);
            double sc = 0.0, sa = 0.0;
            if (A.comp > 0 && B.comp > 0) sc = (double)std::min(A.comp, B.comp) / (double)std::max(A.comp, B.comp);
            if (A.age > 0 && B.age > 0) sa = (double)std::min(A.age, B.age) / (double)std::max(A.age, B.age);
            fv[2]->push_back(sc);
            fv[3]->push_back(sa);
            fv[4]->push_back(region_sim(A.reg, B.reg));
            fv[5]->push_back(set_sim(A.clubs, B.clubs));
            fv[6]->push_back(set_sim(A.friends, B.friends));
            for (size_t t = 0; t < T; ++t)
                text[t].push_back(count_cosine(A.tok.data() + A.col_off[t], A.col_off[t + 1] - A.col_off[t],
                                               B.tok.data() + B.col_off[t], B.col_off[t + 1] - B.col_off[t]));
        }
        for (auto& kv : field) result[kv.first] = mean_sd(kv.second);
        for (size_t t = 0; t < T; ++t) result[ds->cols[t]] = mean_sd(text[t]);
    }
    for (size_t k = 0; k < kFixed + T; ++k) {
        auto it = result.find(k < (size_t)kFixed ? std::string(keys[k]) : ds->cols[k - kFixed]);
        const std::pair<float, float> v = it == result.end() ? std::pair<float, float>(0.0f, 0.0f) : it->second;
        if (out_mean) out_mean[k] = v.first;
        if (out_sd) out_sd[k] = v.second;
    }
    if (save_csv) {  // save_column_normalizers (utils.cpp:144-153)
        std::ofstream out(save_csv);
        if (!out.is_open()) return fail(std::string("cannot write ") + save_csv);
        out << "column,mean,stddev\n";
        for (auto& kv : result) out << kv.first << "," << kv.second.first << "," << kv.second.second << "\n";
    }
    return PF_OK;
}

// ---------------------------------------------------------------- hold-out drivers (A19)

namespace {

struct Topk {
    std::vector<int32_t> uid;
    std::vector<float> score;
    int32_t n = 0;
    explicit Topk(int k) : uid(std::max(k, 1)), score(std::max(k, 1)) {}
};

// run_friends_holdout_test (test.cpp:13-105); adj_mod accumulates over users.  digest (may be
// null): per tested user the pf_result_digest of its collaborative list.
int holdout_friends(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, double* out_ratios, uint64_t* digest,
                    int32_t cap, int32_t* n_out) {
    if (!ctx || !ds || !n_out || (cap > 0 && !out_ratios && !digest)) return PF_EINVAL;
    *n_out = 0;
    std::vector<int> candidates;
    for (auto& kv : ds->profiles) {
        auto it = ds->adj_list.find(kv.first);
        if (it == ds->adj_list.end()) continue;
        if ((int)it->second.size() >= 20) candidates.push_back(kv.first);
    }
    if (candidates.empty()) return PF_OK;
    std::mt19937 rng(1234567);
    std::shuffle(candidates.begin(), candidates.end(), rng);
    std::vector<int> touched;
    std::vector<double> results;
    int taken = 0, rc = PF_OK;
    for (int uid : candidates) {
        if (taken >= sample_size) break;
        const std::vector<int>& friends = ds->adj_list.find(uid)->second;
        const int F = (int)friends.size();
        if (F < 2) continue;
        const int hold_k = F / 5;
        if (hold_k <= 0) continue;
        std::vector<int> idx(F);
        for (int i = 0; i < F; ++i) idx[i] = i;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::unordered_set<int> held;
        for (int i = 0; i < hold_k; ++i) held.insert(friends[idx[i]]);
        std::vector<int32_t> newf;
        newf.reserve(F - hold_k);
        for (int f : friends)
            if (held.find(f) == held.end()) newf.push_back(f);
        rc = pf_set_adj(ctx, uid, newf.data(), (int32_t)newf.size());
        if (rc != PF_OK) break;
        touched.push_back(uid);
        Topk t(hold_k);
        const int32_t q = uid;
        rc = pf_recommend_collab(ctx, &q, 1, hold_k, 1000, t.uid.data(), t.score.data(), &t.n);
        if (rc != PF_OK) break;
        int hits = 0;
        for (int i = 0; i < t.n && i < hold_k; ++i)
            if (held.find(t.uid[i]) != held.end()) ++hits;
        if (digest && taken < cap) digest[taken] = pf_result_digest(t.uid.data(), t.score.data(), t.n);
        results.push_back((double)hits / (double)hold_k);
        ++taken;
    }
    for (int u : touched) {  // the reference mutated a copy (adj_mod); restore the base rows
        const std::vector<int>& f = ds->adj_list.find(u)->second;
        const int r2 = pf_set_adj(ctx, u, f.data(), (int32_t)f.size());
        if (rc == PF_OK) rc = r2;
    }
    if (rc != PF_OK) return rc;
    const int32_t n = (int32_t)results.size();
    for (int32_t i = 0; i < n && i < cap && out_ratios; ++i) out_ratios[i] = results[i];
    *n_out = n;
    return PF_OK;
}

// run_recommendation_tests_sample (recommendation_tests.cpp:68-169); a fresh adj_mod per user.
// digest (may be null): per tested user i, digest[4i .. 4i+3] = pf_result_digest of its graph,
// collaborative, interest and clubs lists; *n_out = users tested.
int recommendation_tests(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk, double* out5,
                         uint64_t* digest, int32_t cap, int32_t* n_out) {
    double scratch[5];
    if (!out5) out5 = scratch;
    for (int i = 0; i < 5; ++i) out5[i] = 0.0;
    if (n_out) *n_out = 0;
    if (ds->profiles.empty() || ds->adj_list.empty()) return PF_OK;
    std::vector<int> all;
    for (auto& kv : ds->profiles) all.push_back(kv.first);
    std::mt19937 rng(1234567);
    std::shuffle(all.begin(), all.end(), rng);
    int taken = 0, hits_graph = 0, hits_collab = 0, hits_interest = 0, club_users = 0;
    double club_prec = 0.0, club_rec = 0.0;
    const int K = std::max(topk, 1);
    for (int uid : all) {
        if (taken >= sample_size) break;
        auto itadj = ds->adj_list.find(uid);
        if (itadj == ds->adj_list.end()) continue;
        const std::vector<int>& friends = itadj->second;
        if (friends.size() < 4) continue;
        const int hold_k = std::max(1, (int)friends.size() / 4);
        std::vector<int> idx(friends.size());
        for (size_t i = 0; i < friends.size(); ++i) idx[i] = (int)i;
        std::shuffle(idx.begin(), idx.end(), rng);
        std::unordered_set<int> held;
        for (int i = 0; i < hold_k; ++i) held.insert(friends[idx[i]]);
        std::vector<int32_t> newf;
        for (int f : friends)
            if (held.find(f) == held.end()) newf.push_back(f);
        int rc = pf_set_adj(ctx, uid, newf.data(), (int32_t)newf.size());
        if (rc != PF_OK) return rc;
        const int32_t q = uid;
        Topk g(K), c(K), in(K), cl(K);
        rc = pf_recommend_interest(ctx, &q, 1, topk, PF_MODE_FOF, 5000, g.uid.data(), g.score.data(), &g.n);
        if (rc == PF_OK) rc = pf_recommend_collab(ctx, &q, 1, topk, 5000, c.uid.data(), c.score.data(), &c.n);
        // recommend_by_interest is recommend_graph_registration (recommender_graph.cpp:224-227)
        in = g;
        if (rc == PF_OK) rc = pf_recommend_clubs(ctx, &q, 1, topk, 5000, cl.uid.data(), cl.score.data(), &cl.n);
        const int r2 = pf_set_adj(ctx, uid, friends.data(), (int32_t)friends.size());
        if (rc != PF_OK) return rc;
        if (r2 != PF_OK) return r2;
        if (digest && taken < cap) {
            uint64_t* d = digest + 4 * (size_t)taken;
            d[0] = pf_result_digest(g.uid.data(), g.score.data(), g.n);
            d[1] = pf_result_digest(c.uid.data(), c.score.data(), c.n);
            d[2] = pf_result_digest(in.uid.data(), in.score.data(), in.n);
            d[3] = pf_result_digest(cl.uid.data(), cl.score.data(), cl.n);
        }
        auto any_held = [&](const Topk& t) {
            for (int i = 0; i < t.n; ++i)
                if (held.find(t.uid[i]) != held.end()) return true;
            return false;
        };
        hits_graph += any_held(g);
        hits_collab += any_held(c);
        hits_interest += any_held(in);
        const auto& row = ds->rows[ds->profiles.find(uid)->second];
        std::unordered_set<int> actual;
        for (uint32_t x : row.clubs) actual.insert((int)x);
        if (!actual.empty()) {
            int hit = 0;
            for (int i = 0; i < cl.n && i < topk; ++i)
                if (actual.find(cl.uid[i]) != actual.end()) ++hit;
            club_prec += (double)hit / (double)topk;
            club_rec += (double)hit / (double)actual.size();
            ++club_users;
        }
        ++taken;
    }
    if (taken > 0) {
        out5[0] = (double)hits_graph / (double)taken;
        out5[1] = (double)hits_collab / (double)taken;
        out5[2] = (double)hits_interest / (double)taken;
    }
    if (club_users > 0) {
        out5[3] = club_prec / (double)club_users;
        out5[4] = club_rec / (double)club_users;
    }
    if (n_out) *n_out = taken;
    return PF_OK;
}

}  // namespace

extern "C" {

int pf_holdout_friends(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, double* out_ratios, int32_t cap,
                       int32_t* n_out) {
    return holdout_friends(ctx, ds, sample_size, out_ratios, nullptr, cap, n_out);
}

int pf_recommendation_tests(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk, double* out5) {
    if (!ctx || !ds || !out5) return PF_EINVAL;
    return recommendation_tests(ctx, ds, sample_size, topk, out5, nullptr, 0, nullptr);
}

int pf_holdout_friends_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, uint64_t* out_digest,
                              int32_t cap, int32_t* n_out) {
    return holdout_friends(ctx, ds, sample_size, nullptr, out_digest, cap, n_out);
}

int pf_recommendation_tests_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk,
                                   uint64_t* out_digest, int32_t cap, int32_t* n_out) {
    if (!ctx || !ds || !n_out || (cap > 0 && !out_digest)) return PF_EINVAL;
    return recommendation_tests(ctx, ds, sample_size, topk, nullptr, out_digest, cap, n_out);
}

}  // extern "C"

// ---------------------------------------------------------------- batched, sharded drivers (F1)
// The sequential drivers above mutate the engine's adjacency between users, so one user runs
// at a time.  Their plans (sampled users, held-out friends) depend only on the rng stream, so
// they are computed up front here; every user's query then reads its adjacency through a view
// (pf_batch.h) and users run in batches (one GPU pair launch per stage), sharded over ranks.

namespace {

struct PlanEntry {
    int32_t uid = 0;
    int hold_k = 0;
    std::vector<int32_t> newf;
    std::unordered_set<int> held;
};

using Plan = std::vector<PlanEntry>;

template <class F>
std::shared_ptr<const Plan> cached_plan(const pf_dataset* ds, int driver, int32_t sample_size, F build) {
    std::lock_guard<std::mutex> g(ds->plan_mu);
    auto& slot = ds->plans[((int64_t)driver << 32) | (uint32_t)sample_size];
    if (!slot) slot = std::make_shared<const Plan>(build());
    return std::static_pointer_cast<const Plan>(slot);
}

// test.cpp:13-60 (candidates with >= 20 friends, shuffled; hold F/5 per user)
std::vector<PlanEntry> plan_friends(const pf_dataset* ds, int32_t sample_size) {
    std::vector<PlanEntry> plan;
    std::vector<int> candidates;
    for (auto& kv : ds->profiles) {
        auto it = ds->adj_list.find(kv.first);
        if (it == ds->adj_list.end()) continue;
        if ((int)it->second.size() >= 20) candidates.push_back(kv.first);
    }
    if (candidates.empty()) return plan;
    std::mt19937 rng(1234567);
    std::shuffle(candidates.begin(), candidates.end(), rng);
    for (int uid : candidates) {
        if ((int32_t)plan.size() >= sample_size) break;
        const std::vector<int>& friends = ds->adj_list.find(uid)->second;
        const int F = (int)friends.size();
        if (F < 2) continue;
        const int hold_k = F / 5;
        if (hold_k <= 0) continue;
        std::vector<int> idx(F);
        for (int i = 0; i < F; ++i) idx[i] = i;
        std::shuffle(idx.begin(), idx.end(), rng);
        PlanEntry e;
        e.uid = uid;
        e.hold_k = hold_k;
        for (int i = 0; i < hold_k; ++i) e.held.insert(friends[idx[i]]);
        for (int f : friends)
            if (e.held.find(f) == e.held.end()) e.newf.push_back(f);
        plan.push_back(std::move(e));
    }
    return plan;
}

// recommendation_tests.cpp:76-115 (all profiles shuffled; degree >= 4; hold max(1, F/4))
std::vector<PlanEntry> plan_rec(const pf_dataset* ds, int32_t sample_size) {
    std::vector<PlanEntry> plan;
    if (ds->profiles.empty() || ds->adj_list.empty()) return plan;
    std::vector<int> all;
    for (auto& kv : ds->profiles) all.push_back(kv.first);
    std::mt19937 rng(1234567);
    std::shuffle(all.begin(), all.end(), rng);
    for (int uid : all) {
        if ((int32_t)plan.size() >= sample_size) break;
        auto itadj = ds->adj_list.find(uid);
        if (itadj == ds->adj_list.end()) continue;
        const std::vector<int>& friends = itadj->second;
        if (friends.size() < 4) continue;
        const int hold_k = std::max(1, (int)friends.size() / 4);
        std::vector<int> idx(friends.size());
        for (size_t i = 0; i < friends.size(); ++i) idx[i] = (int)i;
        std::shuffle(idx.begin(), idx.end(), rng);
        PlanEntry e;
        e.uid = uid;
        e.hold_k = hold_k;
        for (int i = 0; i < hold_k; ++i) e.held.insert(friends[idx[i]]);
        for (int f : friends)
            if (e.held.find(f) == e.held.end()) e.newf.push_back(f);
        plan.push_back(std::move(e));
    }
    return plan;
}

// The versioned edit set of a driver call lives on the call's stack: the engine forgets it when
// the call starts and ends (pf_jobs_plan.cpp jobs_view_scope).
struct ViewScope {
    pf_ctx* c;
    explicit ViewScope(pf_ctx* x) : c(x) { pf::jobs_view_scope(c); }
    ~ViewScope() { pf::jobs_view_scope(c); }
};

bool bad_shard(int32_t shard, int32_t nshards, int32_t batch) {
    return nshards < 1 || shard < 0 || shard >= nshards || batch < 1;
}

uint64_t job_digest(const pf::Job& J) {
    std::vector<int32_t> ids;
    std::vector<float> sc;
    for (const auto& kv : J.out) {
        ids.push_back(kv.first);
        sc.push_back(kv.second);
    }
    return pf_result_digest(ids.data(), sc.data(), (int32_t)ids.size());
}

int eval_holdout_friends(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t shard, int32_t nshards,
                         int32_t batch, double* out_ratio, uint64_t* digest, int32_t cap, int32_t* n_plan) {
    if (!ctx || !ds || !n_plan || (cap > 0 && !out_ratio && !digest) || bad_shard(shard, nshards, batch))
        return PF_EINVAL;
    pf::HpLap hl;
    ViewScope scope(ctx);
    const auto planp = cached_plan(ds, 0, sample_size, [&]() { return plan_friends(ds, sample_size); });
    const Plan& plan = *planp;
    hl.lap(pf::kHpPlan);
    *n_plan = (int32_t)plan.size();
    // one adj_mod for the whole run (test.cpp:35,73): user i sees the rows of users 0..i edited
    std::unordered_map<int32_t, std::pair<int32_t, std::vector<int32_t>>> over;
    for (size_t i = 0; i < plan.size(); ++i) over[plan[i].uid] = {(int32_t)i, plan[i].newf};
    const auto& base = pf::base_adj(ctx);
    std::vector<int32_t> mine;
    for (int32_t i = shard; i < (int32_t)plan.size(); i += nshards) mine.push_back(i);
    for (size_t b = 0; b < mine.size(); b += (size_t)batch) {
        const size_t e = std::min(mine.size(), b + (size_t)batch);
        std::vector<pf::Job> jobs(e - b);
        for (size_t x = b; x < e; ++x) {
            const PlanEntry& pe = plan[mine[x]];
            pf::Job& J = jobs[x - b];
            J.kind = pf::kJobCollab;
            J.uid = pe.uid;
            J.topk = pe.hold_k;
            J.limit = 1000;  // test.cpp:75
            J.view.base = &base;
            J.view.over = &over;
            J.view.version = mine[x];
        }
        const int rc = pf::run_jobs(ctx, jobs);
        if (rc != PF_OK) return rc;
        for (size_t x = b; x < e; ++x) {
            const PlanEntry& pe = plan[mine[x]];
            const auto& out = jobs[x - b].out;
            int hits = 0;
            for (int i = 0; i < (int)out.size() && i < pe.hold_k; ++i)
                if (pe.held.find(out[i].first) != pe.held.end()) ++hits;
            if (mine[x] >= cap) continue;
            if (out_ratio) out_ratio[mine[x]] = (double)hits / (double)pe.hold_k;
            if (digest) digest[mine[x]] = job_digest(jobs[x - b]);
        }
    }
    return PF_OK;
}

// The carried call's hold on its dataset (pf_dataset::holds): released when the call's closure is
// destroyed (finished, failed or dropped by pf_close), deleting a dataset freed meanwhile.
struct DsHold {
    pf_dataset* ds;
    explicit DsHold(const pf_dataset* d) : ds(const_cast<pf_dataset*>(d)) {
        std::lock_guard<std::mutex> g(ds->hold_mu);
        ++ds->holds;
    }
    ~DsHold() {
        bool del = false;
        {
            std::lock_guard<std::mutex> g(ds->hold_mu);
            del = --ds->holds == 0 && ds->free_pending;
        }
        if (del) delete ds;
    }
    DsHold(const DsHold&) = delete;
    DsHold& operator=(const DsHold&) = delete;
};

int eval_recommendation_tests(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk, int32_t shard,
                              int32_t nshards, int32_t batch, int8_t* out_hits, double* out_club, uint64_t* digest,
                              int32_t cap, int32_t* n_plan, uint64_t* ticket = nullptr) {
    if (!ctx || !ds || !n_plan || (cap > 0 && !digest && (!out_hits || !out_club)) || bad_shard(shard, nshards, batch))
        return PF_EINVAL;
    pf::HpLap hl;
    ViewScope scope(ctx);
    const auto planp = cached_plan(ds, 1, sample_size, [&]() { return plan_rec(ds, sample_size); });
    hl.lap(pf::kHpPlan);
    *n_plan = (int32_t)planp->size();
    const auto& base = pf::base_adj(ctx);
    auto mine = std::make_shared<std::vector<int32_t>>();
    for (int32_t i = shard; i < (int32_t)planp->size(); i += nshards) mine->push_back(i);
    // the per-user results of plan entries mine[b .. e) from their finished jobs (3 per user);
    // everything it reads is captured by value, so a carried call can run it later
    auto score = [planp, mine, ds, topk, out_hits, out_club, digest, cap](std::vector<pf::Job>& jobs, size_t b,
                                                                          size_t e) {
        const Plan& plan = *planp;
        for (size_t x = b; x < e; ++x) {
            const int32_t i = (*mine)[x];
            if (i >= cap) continue;
            const PlanEntry& pe = plan[i];
            auto any_held = [&](const pf::Job& J) {
                for (auto& kv : J.out)
                    if (pe.held.find(kv.first) != pe.held.end()) return true;
                return false;
            };
            const pf::Job& g = jobs[3 * (x - b)];
            if (digest) {
                uint64_t* d = digest + 4 * (size_t)i;
                d[0] = d[2] = job_digest(g);  // recommend_by_interest = recommend_graph_registration
                d[1] = job_digest(jobs[3 * (x - b) + 1]);
                d[3] = job_digest(jobs[3 * (x - b) + 2]);
            }
            if (!out_hits) continue;
            out_hits[3 * (size_t)i] = (int8_t)any_held(g);
            out_hits[3 * (size_t)i + 1] = (int8_t)any_held(jobs[3 * (x - b) + 1]);
            out_hits[3 * (size_t)i + 2] = (int8_t)any_held(g);
            const auto& row = ds->rows[ds->profiles.find(pe.uid)->second];
            std::unordered_set<int> actual;
            for (uint32_t c : row.clubs) actual.insert((int)c);
            out_club[2 * (size_t)i] = NAN;
            out_club[2 * (size_t)i + 1] = NAN;
            if (!actual.empty()) {
                const auto& cl = jobs[3 * (x - b) + 2].out;
                int hit = 0;
                for (int j = 0; j < (int)cl.size() && j < topk; ++j)
                    if (actual.find(cl[j].first) != actual.end()) ++hit;
                out_club[2 * (size_t)i] = (double)hit / (double)topk;
                out_club[2 * (size_t)i + 1] = (double)hit / (double)actual.size();
            }
        }
    };
    for (size_t b = 0; b < mine->size(); b += (size_t)batch) {
        const size_t e = std::min(mine->size(), b + (size_t)batch);
        // per user: graph (= interest, recommender_graph.cpp:224-227), collaborative, clubs; limit 5000
        std::vector<pf::Job> jobs(3 * (e - b));
        for (size_t x = b; x < e; ++x) {
            const PlanEntry& pe = (*planp)[(*mine)[x]];
            for (int kind = 0; kind < 3; ++kind) {
                pf::Job& J = jobs[3 * (x - b) + kind];
                J.kind = kind == 0 ? pf::kJobInterest : (kind == 1 ? pf::kJobCollab : pf::kJobClubs);
                J.uid = pe.uid;
                J.topk = topk;
                J.limit = 5000;
                J.view.base = &base;  // a fresh adj_mod per user: only its own row edited
                J.view.own = pe.uid;
                J.view.own_row = &pe.newf;
            }
        }
        if (ticket && e == mine->size()) {  // the last batch stays on the device (its results: pf_wait)
            auto hold = std::make_shared<DsHold>(ds);  // ds outlives the carried call (pf_dataset_free defers)
            return pf::run_jobs_carry(ctx, std::move(jobs), *ticket,
                                      [score, b, e, hold](std::vector<pf::Job>& js) { score(js, b, e); });
        }
        const int rc = pf::run_jobs(ctx, jobs);
        if (rc != PF_OK) return rc;
        score(jobs, b, e);
    }
    return PF_OK;
}

}  // namespace

extern "C" {

int pf_eval_holdout_friends(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t shard, int32_t nshards,
                            int32_t batch, double* out_ratio, int32_t cap, int32_t* n_plan) {
    if (cap > 0 && !out_ratio) return PF_EINVAL;
    return eval_holdout_friends(ctx, ds, sample_size, shard, nshards, batch, out_ratio, nullptr, cap, n_plan);
}

int pf_eval_recommendation_tests(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk, int32_t shard,
                                 int32_t nshards, int32_t batch, int8_t* out_hits, double* out_club, int32_t cap,
                                 int32_t* n_plan) {
    if (cap > 0 && (!out_hits || !out_club)) return PF_EINVAL;
    return eval_recommendation_tests(ctx, ds, sample_size, topk, shard, nshards, batch, out_hits, out_club, nullptr,
                                     cap, n_plan);
}

int pf_eval_holdout_friends_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t shard,
                                   int32_t nshards, int32_t batch, uint64_t* out_digest, int32_t cap, int32_t* n_plan) {
    if (cap > 0 && !out_digest) return PF_EINVAL;
    return eval_holdout_friends(ctx, ds, sample_size, shard, nshards, batch, nullptr, out_digest, cap, n_plan);
}

int pf_eval_recommendation_tests_async(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk,
                                       int32_t shard, int32_t nshards, int32_t batch, int8_t* out_hits,
                                       double* out_club, int32_t cap, int32_t* n_plan, uint64_t* ticket) {
    if (!ticket || (cap > 0 && (!out_hits || !out_club))) return PF_EINVAL;
    if (!ctx) return PF_EINVAL;
    *ticket = pf::next_call_ticket(ctx);
    return eval_recommendation_tests(ctx, ds, sample_size, topk, shard, nshards, batch, out_hits, out_club, nullptr,
                                     cap, n_plan, ticket);
}

int pf_eval_recommendation_tests_digest(pf_ctx* ctx, const pf_dataset* ds, int32_t sample_size, int32_t topk,
                                        int32_t shard, int32_t nshards, int32_t batch, uint64_t* out_digest,
                                        int32_t cap, int32_t* n_plan) {
    if (cap > 0 && !out_digest) return PF_EINVAL;
    return eval_recommendation_tests(ctx, ds, sample_size, topk, shard, nshards, batch, nullptr, nullptr, out_digest,
                                     cap, n_plan);
}

}  // extern "C"
