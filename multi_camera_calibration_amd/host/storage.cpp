// storage.cpp -- cv::FileStorage subset (include/mcc_storage.hpp): XML / YAML read and write of
// ints, reals, strings, opencv-matrix nodes and sequences of them.
#include "mcc_storage.hpp"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace mcc {
namespace storage {

namespace {

[[noreturn]] void bad(const std::string& path, const std::string& what) {
    throw std::runtime_error("FileStorage " + path + ": " + what);
}

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

std::string unquote(std::string s) {
    s = trim(s);
    if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\'')))
        return s.substr(1, s.size() - 2);
    return s;
}

// "3d" -> channels 3, depth 'd'
void parse_dt(const std::string& dt0, int& ch, char& depth) {
    const std::string dt = unquote(dt0);
    size_t i = 0;
    ch = 0;
    while (i < dt.size() && std::isdigit((unsigned char)dt[i])) ch = ch * 10 + (dt[i++] - '0');
    if (ch == 0) ch = 1;
    if (i >= dt.size()) throw std::runtime_error("bad dt '" + dt0 + "'");
    depth = dt[i];
}

std::vector<double> parse_numbers(const std::string& s) {
    std::vector<double> v;
    const char* p = s.c_str();
    while (*p) {
        while (*p && (std::isspace((unsigned char)*p) || *p == ',' || *p == '[' || *p == ']')) ++p;
        if (!*p) break;
        char* end = nullptr;
        const double x = std::strtod(p, &end);
        if (end == p) throw std::runtime_error(std::string("bad number near '") + std::string(p).substr(0, 20) + "'");
        v.push_back(x);
        p = end;
    }
    return v;
}

Node scalar_node(const std::string& text) {
    Node n;
    const std::string t = trim(text);
    if (!t.empty() && t.front() == '"') {
        n.type = Node::STRING;
        n.str = unquote(t);
        return n;
    }
    char* end = nullptr;
    const long long iv = std::strtoll(t.c_str(), &end, 10);
    if (!t.empty() && *end == '\0') {
        n.type = Node::INT;
        n.integer = iv;
        n.real = (double)iv;
        return n;
    }
    const double rv = std::strtod(t.c_str(), &end);
    if (!t.empty() && *end == '\0') {
        n.type = Node::REAL;
        n.real = rv;
        return n;
    }
    n.type = Node::STRING;
    n.str = t;
    return n;
}

// a whitespace / comma separated list ('[' ']' allowed) of numbers, or of (quoted) strings such as
// imagelist_creator's image names: REAL nodes when every token is a number, STRING nodes otherwise
Node list_node(const std::string& text) {
    std::vector<std::string> toks;
    std::string cur;
    bool quoted = false;
    for (char c : text) {
        if (c == '"') {
            quoted = !quoted;
            cur += c;
        } else if (!quoted && (std::isspace((unsigned char)c) || c == ',' || c == '[' || c == ']')) {
            if (!cur.empty()) toks.push_back(cur);
            cur.clear();
        } else {
            cur += c;
        }
    }
    if (!cur.empty()) toks.push_back(cur);
    bool numeric = true;
    for (const std::string& t : toks) {
        char* end = nullptr;
        std::strtod(t.c_str(), &end);
        numeric = numeric && end && *end == '\0' && !t.empty();
    }
    Node n;
    n.type = Node::SEQ;
    for (const std::string& t : toks) {
        Node k;
        if (numeric) {
            k.type = Node::REAL;
            k.real = std::strtod(t.c_str(), nullptr);
        } else {
            k.type = Node::STRING;
            k.str = unquote(t);
        }
        n.seq.push_back(k);
    }
    return n;
}

Node make_mat(int rows, int cols, const std::string& dt, const std::string& data) {
    Node n;
    n.type = Node::MAT;
    Mat& m = n.mat;
    m.rows = rows;
    m.cols = cols;
    parse_dt(dt, m.channels, m.depth);
    m.data = parse_numbers(data);
    if (m.depth == 'f')   // stored as float (CV_32F), as cv::FileStorage reads it
        for (double& v : m.data) v = (double)(float)v;
    if (m.data.size() != (size_t)rows * cols * m.channels)
        throw std::runtime_error("matrix data has " + std::to_string(m.data.size()) + " values, expected " +
                                 std::to_string((size_t)rows * cols * m.channels));
    return n;
}

// ---------------------------------------------------------------- XML
struct XmlElem {
    std::string name;
    std::map<std::string, std::string> attr;
    std::string text;
    std::vector<XmlElem> kids;
};

class XmlParser {
public:
    explicit XmlParser(const std::string& s) : s_(s) {}
    XmlElem root() {
        skip_misc();
        XmlElem e = element();
        return e;
    }

private:
    const std::string& s_;
    size_t p_ = 0;
    void ws() {
        while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
    }
    void skip_misc() {   // <?xml ... ?>, <!-- ... -->
        for (;;) {
            ws();
            if (s_.compare(p_, 2, "<?") == 0) {
                const size_t q = s_.find("?>", p_);
                if (q == std::string::npos) throw std::runtime_error("unterminated <?");
                p_ = q + 2;
            } else if (s_.compare(p_, 4, "<!--") == 0) {
                const size_t q = s_.find("-->", p_);
                if (q == std::string::npos) throw std::runtime_error("unterminated comment");
                p_ = q + 3;
            } else {
                return;
            }
        }
    }
    XmlElem element() {
        if (p_ >= s_.size() || s_[p_] != '<') throw std::runtime_error("expected '<'");
        ++p_;
        XmlElem e;
        while (p_ < s_.size() && !std::isspace((unsigned char)s_[p_]) && s_[p_] != '>' && s_[p_] != '/') e.name += s_[p_++];
        for (;;) {   // attributes
            ws();
            if (p_ >= s_.size()) throw std::runtime_error("unterminated tag " + e.name);
            if (s_[p_] == '/') {   // <name/>
                p_ += 2;
                return e;
            }
            if (s_[p_] == '>') {
                ++p_;
                break;
            }
            std::string k;
            while (p_ < s_.size() && s_[p_] != '=' && !std::isspace((unsigned char)s_[p_])) k += s_[p_++];
            ws();
            if (s_[p_] != '=') throw std::runtime_error("bad attribute in " + e.name);
            ++p_;
            ws();
            const char q = s_[p_++];
            const size_t end = s_.find(q, p_);
            if (end == std::string::npos) throw std::runtime_error("unterminated attribute in " + e.name);
            e.attr[k] = s_.substr(p_, end - p_);
            p_ = end + 1;
        }
        for (;;) {   // content
            const size_t lt = s_.find('<', p_);
            if (lt == std::string::npos) throw std::runtime_error("unterminated element " + e.name);
            e.text += s_.substr(p_, lt - p_);
            p_ = lt;
            if (s_.compare(p_, 4, "<!--") == 0) {
                skip_misc();
                continue;
            }
            if (s_.compare(p_, 2, "</") == 0) {
                const size_t gt = s_.find('>', p_);
                const std::string nm = trim(s_.substr(p_ + 2, gt - p_ - 2));
                if (nm != e.name) throw std::runtime_error("mismatched </" + nm + "> for <" + e.name + ">");
                p_ = gt + 1;
                return e;
            }
            e.kids.push_back(element());
        }
    }
};

Node xml_node(const XmlElem& e) {
    auto it = e.attr.find("type_id");
    if (it != e.attr.end() && it->second == "opencv-matrix") {
        std::map<std::string, std::string> f;
        for (const XmlElem& k : e.kids) f[k.name] = k.text;
        if (!f.count("rows") || !f.count("cols") || !f.count("dt") || !f.count("data"))
            throw std::runtime_error("incomplete opencv-matrix " + e.name);
        return make_mat(std::atoi(f["rows"].c_str()), std::atoi(f["cols"].c_str()), f["dt"], f["data"]);
    }
    if (!e.kids.empty()) {
        Node n;
        n.type = Node::SEQ;
        for (const XmlElem& k : e.kids) n.seq.push_back(xml_node(k));
        return n;
    }
    const std::string t = trim(e.text);
    if (t.find_first_of(" \n\t") != std::string::npos && !(t.front() == '"' && t.back() == '"' &&
                                                          t.find('"', 1) == t.size() - 1))
        return list_node(t);   // a whitespace-separated list of numbers or strings
    return scalar_node(t);
}

// ---------------------------------------------------------------- YAML (OpenCV's subset)
struct YLine {
    int indent;
    std::string text;
};

class YamlParser {
public:
    explicit YamlParser(const std::string& s) {
        std::istringstream in(s);
        std::string line;
        while (std::getline(in, line)) {
            if (!line.empty() && line.back() == '\r') line.pop_back();
            const std::string t = trim(line);
            if (t.empty() || t[0] == '#' || t[0] == '%' || t == "---" || t == "...") continue;
            int ind = 0;
            while (ind < (int)line.size() && line[ind] == ' ') ++ind;
            lines_.push_back({ind, t});
        }
    }
    std::map<std::string, Node> top(std::vector<std::string>& order) {
        std::map<std::string, Node> out;
        while (i_ < lines_.size()) {
            const YLine& l = lines_[i_];
            std::string key, rest;
            split_key(l.text, key, rest);
            ++i_;
            out[key] = value(rest, l.indent);
            order.push_back(key);
        }
        return out;
    }

private:
    std::vector<YLine> lines_;
    size_t i_ = 0;

    static void split_key(const std::string& t, std::string& key, std::string& rest) {
        const size_t c = t.find(':');
        if (c == std::string::npos) throw std::runtime_error("expected 'key: value' in '" + t + "'");
        key = unquote(t.substr(0, c));
        rest = trim(t.substr(c + 1));
    }
    // a '[' ... ']' list possibly spanning lines
    std::string bracket(std::string first) {
        std::string acc = first;
        while (acc.find(']') == std::string::npos) {
            if (i_ >= lines_.size()) throw std::runtime_error("unterminated '['");
            acc += " " + lines_[i_++].text;
        }
        return acc;
    }
    Node mapping_mat(int parent_indent) {
        std::map<std::string, std::string> f;
        while (i_ < lines_.size() && lines_[i_].indent > parent_indent && lines_[i_].text[0] != '-') {
            std::string k, r;
            split_key(lines_[i_].text, k, r);
            ++i_;
            if (k == "data") r = bracket(r);
            f[k] = r;
        }
        if (!f.count("rows") || !f.count("cols") || !f.count("dt") || !f.count("data"))
            throw std::runtime_error("incomplete opencv-matrix");
        return make_mat(std::atoi(f["rows"].c_str()), std::atoi(f["cols"].c_str()), f["dt"], f["data"]);
    }
    Node value(const std::string& rest, int indent) {
        if (rest.rfind("!!opencv-matrix", 0) == 0) return mapping_mat(indent);
        if (!rest.empty() && rest[0] == '[') return list_node(bracket(rest));
        if (!rest.empty()) return scalar_node(rest);
        // block sequence: "- item" lines deeper than (or at) the key's indent
        Node n;
        n.type = Node::SEQ;
        while (i_ < lines_.size() && lines_[i_].text[0] == '-' && lines_[i_].indent >= indent) {
            const int ind = lines_[i_].indent;
            const std::string item = trim(lines_[i_].text.substr(1));
            ++i_;
            n.seq.push_back(value(item, ind));
        }
        return n;
    }
};

// ---------------------------------------------------------------- writers
std::string num(double v, char depth) {
    char b[64];
    if (depth != 'f' && depth != 'd') {
        std::snprintf(b, sizeof b, "%lld", (long long)v);
    } else if (v == std::floor(v) && std::fabs(v) < 1e9) {
        std::snprintf(b, sizeof b, "%lld.", (long long)v);
    } else {
        std::snprintf(b, sizeof b, depth == 'f' ? "%.8e" : "%.16e", v);
    }
    return b;
}

std::string dt_string(const Mat& m, bool quote) {
    std::string s = (m.channels > 1 ? std::to_string(m.channels) : std::string()) + m.depth;
    return (quote && m.channels > 1) ? "\"" + s + "\"" : s;
}

}  // namespace

double Node::toReal() const {
    if (type == INT) return (double)integer;
    if (type == REAL) return real;
    throw std::runtime_error("FileStorage node is not a number");
}
int Node::toInt() const {
    if (type == INT) return (int)integer;
    if (type == REAL) return (int)std::lround(real);
    throw std::runtime_error("FileStorage node is not a number");
}

std::string resolve_path(const std::string& path) {
    const char* env = std::getenv("MCC_PATH_MAP");
    if (!env || !*env) return path;
    const std::string map(env);
    size_t pos = 0;
    while (pos <= map.size()) {
        size_t end = map.find(';', pos);
        if (end == std::string::npos) end = map.size();
        const std::string item = map.substr(pos, end - pos);
        const size_t eq = item.find('=');
        if (eq != std::string::npos && eq > 0) {
            const std::string from = item.substr(0, eq), to = item.substr(eq + 1);
            if (path.compare(0, from.size(), from) == 0) return to + path.substr(from.size());
        }
        pos = end + 1;
    }
    return path;
}

FileStorage::FileStorage(const std::string& path_in, int flags) : path_(resolve_path(path_in)), flags_(flags) {
    const std::string& path = path_;
    xml_ = !(ends_with(path, ".yml") || ends_with(path, ".yaml"));
    if (flags == WRITE) {
        std::ofstream probe(path, std::ios::app);
        opened_ = (bool)probe;
        return;
    }
    std::ifstream in(path, std::ios::binary);
    if (!in) return;
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string s = ss.str();
    const std::string head = trim(s.substr(0, 64));
    try {
        if (head.rfind("%YAML", 0) == 0 || head.rfind("---", 0) == 0) {
            xml_ = false;
            YamlParser y(s);
            nodes_ = y.top(order_);
        } else {
            xml_ = true;
            XmlParser x(s);
            const XmlElem root = x.root();
            if (root.name != "opencv_storage") bad(path, "root element is <" + root.name + ">, not <opencv_storage>");
            for (const XmlElem& k : root.kids) {
                nodes_[k.name] = xml_node(k);
                order_.push_back(k.name);
            }
        }
    } catch (const std::runtime_error& e) {
        bad(path, e.what());
    }
    opened_ = true;
}

FileStorage::~FileStorage() {
    try {
        release();
    } catch (...) {
    }
}

const Node& FileStorage::operator[](const std::string& key) const {
    static const Node none;
    auto it = nodes_.find(key);
    return it == nodes_.end() ? none : it->second;
}

void FileStorage::put(const std::string& key, Node n) {
    if (flags_ != WRITE) bad(path_, "not opened for writing");
    if (!nodes_.count(key)) order_.push_back(key);
    nodes_[key] = std::move(n);
}
void FileStorage::write(const std::string& key, int v) {
    Node n;
    n.type = Node::INT;
    n.integer = v;
    put(key, n);
}
void FileStorage::write(const std::string& key, double v) {
    Node n;
    n.type = Node::REAL;
    n.real = v;
    put(key, n);
}
void FileStorage::write(const std::string& key, const std::string& v) {
    Node n;
    n.type = Node::STRING;
    n.str = v;
    put(key, n);
}
void FileStorage::write(const std::string& key, const Mat& m) {
    Node n;
    n.type = Node::MAT;
    n.mat = m;
    put(key, n);
}

void FileStorage::release() {
    if (flags_ != WRITE || !opened_) return;
    opened_ = false;
    std::ofstream out(path_, std::ios::trunc);
    if (!out) bad(path_, "cannot write");
    if (xml_) {
        out << "<?xml version=\"1.0\"?>\n<opencv_storage>\n";
        for (const std::string& k : order_) {
            const Node& n = nodes_[k];
            if (n.type == Node::MAT) {
                const Mat& m = n.mat;
                out << "<" << k << " type_id=\"opencv-matrix\">\n  <rows>" << m.rows << "</rows>\n  <cols>" << m.cols
                    << "</cols>\n  <dt>" << dt_string(m, true) << "</dt>\n  <data>";
                for (size_t i = 0; i < m.data.size(); ++i) out << ((i % 4 == 0) ? "\n    " : " ") << num(m.data[i], m.depth);
                out << "</data></" << k << ">\n";
            } else if (n.type == Node::INT) {
                out << "<" << k << ">" << n.integer << "</" << k << ">\n";
            } else if (n.type == Node::REAL) {
                out << "<" << k << ">" << num(n.real, 'd') << "</" << k << ">\n";
            } else {
                out << "<" << k << ">\"" << n.str << "\"</" << k << ">\n";
            }
        }
        out << "</opencv_storage>\n";
    } else {
        out << "%YAML:1.0\n---\n";
        for (const std::string& k : order_) {
            const Node& n = nodes_[k];
            if (n.type == Node::MAT) {
                const Mat& m = n.mat;
                out << k << ": !!opencv-matrix\n   rows: " << m.rows << "\n   cols: " << m.cols << "\n   dt: "
                    << dt_string(m, true) << "\n   data: [";
                for (size_t i = 0; i < m.data.size(); ++i)
                    out << (i ? ", " : " ") << ((i && i % 4 == 0) ? "\n       " : "") << num(m.data[i], m.depth);
                out << " ]\n";
            } else if (n.type == Node::INT) {
                out << k << ": " << n.integer << "\n";
            } else if (n.type == Node::REAL) {
                out << k << ": " << num(n.real, 'd') << "\n";
            } else {
                out << k << ": \"" << n.str << "\"\n";
            }
        }
    }
    if (!out) bad(path_, "write failed");
}

}  // namespace storage
}  // namespace mcc
