// yaml.cc — see yaml.h. A line-oriented recursive-descent parser: each logical line carries its
// indentation; block collections are parsed by indentation level, scalars/flow collections by a
// small character scanner.
#include "core/yaml.h"

#include <cctype>
#include <cstdlib>
#include <stdexcept>

namespace kf {
namespace {

struct YamlError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct Line {
  int indent;
  std::string text;  // without indentation, comments stripped (outside quotes)
  int no;            // 1-based source line
};

std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
  }
  return s;
}

std::string rtrim(std::string s) {
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  return s;
}
std::string ltrim(const std::string& s) {
  size_t i = 0;
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
  return s.substr(i);
}

Json resolve_plain(const std::string& s) {
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Json();
  if (s == "true" || s == "True" || s == "TRUE") return Json(true);
  if (s == "false" || s == "False" || s == "FALSE") return Json(false);
  // ints (decimal, 0x, 0o) and floats
  char* end = nullptr;
  if (s.size() > 2 && s[0] == '0' && (s[1] == 'x' || s[1] == 'o')) {
    long long v = std::strtoll(s.c_str() + 2, &end, s[1] == 'x' ? 16 : 8);
    if (*end == 0) return Json(v);
  }
  bool numeric = true, has_digit = false, floaty = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (std::isdigit(static_cast<unsigned char>(c))) has_digit = true;
    else if ((c == '-' || c == '+') && (i == 0 || s[i - 1] == 'e' || s[i - 1] == 'E')) continue;
    else if (c == '.' || c == 'e' || c == 'E') floaty = true;
    else numeric = false;
  }
  if (numeric && has_digit) {
    if (!floaty) {
      long long v = std::strtoll(s.c_str(), &end, 10);
      if (*end == 0) return Json(v);
    } else {
      double d = std::strtod(s.c_str(), &end);
      if (*end == 0) return Json(d);
    }
  }
  if (s == ".inf" || s == ".Inf") return Json(1e308 * 10);
  return Json(s);
}

// ---- flow / scalar scanner ------------------------------------------------------------------------
struct Scanner {
  const std::string& s;
  size_t i = 0;
  int line;
  explicit Scanner(const std::string& str, int ln) : s(str), line(ln) {}
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n')) ++i;
  }
  [[noreturn]] void fail(const std::string& m) { throw YamlError("line " + std::to_string(line) + ": " + m); }
  std::string quoted() {
    char q = s[i++];
    std::string out;
    while (i < s.size()) {
      char c = s[i++];
      if (q == '\'' && c == '\'') {
        if (i < s.size() && s[i] == '\'') {
          out += '\'';
          ++i;
          continue;
        }
        return out;
      }
      if (q == '"' && c == '"') return out;
      if (q == '"' && c == '\\' && i < s.size()) {
        char e = s[i++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case '0': out += '\0'; break;
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case '\n':  // escaped line break: join without a space, drop the next line's indentation
            while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
            break;
          case 'u': {
            unsigned cp = static_cast<unsigned>(std::strtoul(s.substr(i, 4).c_str(), nullptr, 16));
            i += 4;
            if (cp < 0x80) out += static_cast<char>(cp);
            else if (cp < 0x800) {
              out += static_cast<char>(0xC0 | (cp >> 6));
              out += static_cast<char>(0x80 | (cp & 0x3F));
            } else {
              out += static_cast<char>(0xE0 | (cp >> 12));
              out += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
              out += static_cast<char>(0x80 | (cp & 0x3F));
            }
            break;
          }
          default: out += e;
        }
        continue;
      }
      if (c == '\n') {
        // line folding inside quotes
        while (!out.empty() && out.back() == ' ') out.pop_back();
        out += ' ';
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
        continue;
      }
      out += c;
    }
    fail("unterminated quoted scalar");
  }
  // plain scalar in flow context: stops at , ] } and ": "
  std::string plain_flow() {
    size_t st = i;
    while (i < s.size() && s[i] != ',' && s[i] != ']' && s[i] != '}' && !(s[i] == ':' && (i + 1 >= s.size() || s[i + 1] == ' ')))
      ++i;
    return rtrim(s.substr(st, i - st));
  }
  Json value_flow() {
    ws();
    if (i >= s.size()) fail("unexpected end in flow collection");
    if (s[i] == '[') return seq();
    if (s[i] == '{') return map();
    if (s[i] == '"' || s[i] == '\'') return Json(quoted());
    return resolve_plain(plain_flow());
  }
  Json seq() {
    ++i;
    Json out = Json::array();
    ws();
    if (i < s.size() && s[i] == ']') {
      ++i;
      return out;
    }
    while (true) {
      out.push_back(value_flow());
      ws();
      if (i < s.size() && s[i] == ',') {
        ++i;
        ws();
        if (i < s.size() && s[i] == ']') {
          ++i;
          return out;
        }
        continue;
      }
      if (i < s.size() && s[i] == ']') {
        ++i;
        return out;
      }
      fail("expected , or ] in flow sequence");
    }
  }
  Json map() {
    ++i;
    Json out = Json::object();
    ws();
    if (i < s.size() && s[i] == '}') {
      ++i;
      return out;
    }
    while (true) {
      ws();
      std::string key = (s[i] == '"' || s[i] == '\'') ? quoted() : plain_flow();
      ws();
      Json val;
      if (i < s.size() && s[i] == ':') {
        ++i;
        val = value_flow();
      }
      out[key] = val;
      ws();
      if (i < s.size() && s[i] == ',') {
        ++i;
        continue;
      }
      if (i < s.size() && s[i] == '}') {
        ++i;
        return out;
      }
      fail("expected , or } in flow mapping");
    }
  }
};

// ---- block parser -----------------------------------------------------------------------------
class Parser {
 public:
  Parser(const std::vector<std::string>& raw) : raw_(raw) {
    for (size_t n = 0; n < raw.size(); ++n) {
      std::string t = rtrim(strip_comment(raw[n]));
      size_t ind = 0;
      while (ind < t.size() && t[ind] == ' ') ++ind;
      if (ind == t.size()) continue;
      lines_.push_back({static_cast<int>(ind), t.substr(ind), static_cast<int>(n + 1)});
    }
  }
  Json parse() {
    if (lines_.empty()) return Json();
    Json v = block(lines_[0].indent);
    if (pos_ < lines_.size()) throw YamlError("line " + std::to_string(lines_[pos_].no) + ": unexpected content (bad indentation?)");
    return v;
  }

 private:
  [[noreturn]] void fail(int line, const std::string& m) { throw YamlError("line " + std::to_string(line) + ": " + m); }

  static bool is_seq_item(const std::string& t) { return t == "-" || (t.size() > 1 && t[0] == '-' && t[1] == ' '); }

  // position of the mapping ':' separator in a line (outside quotes/flow), or npos
  static size_t key_colon(const std::string& t) {
    if (t.empty() || t[0] == '[' || t[0] == '{') return std::string::npos;
    bool sq = false, dq = false;
    for (size_t i = 0; i < t.size(); ++i) {
      char c = t[i];
      if (c == '\'' && !dq) sq = !sq;
      else if (c == '"' && !sq) dq = !dq;
      else if (c == ':' && !sq && !dq && (i + 1 == t.size() || t[i + 1] == ' ')) return i;
    }
    return std::string::npos;
  }

  Json block(int indent) {
    const Line& l = lines_[pos_];
    if (is_seq_item(l.text)) return sequence(l.indent);
    if (key_colon(l.text) != std::string::npos) return mapping(l.indent);
    // a lone scalar (possibly multi-line plain / flow)
    return scalar_lines(indent);
  }

  Json scalar_lines(int indent) {
    std::string acc;
    int no = lines_[pos_].no;
    while (pos_ < lines_.size() && lines_[pos_].indent >= indent) {
      if (!acc.empty()) acc += (acc[0] == '[' || acc[0] == '{' || acc[0] == '"' || acc[0] == '\'') ? "\n" : " ";
      acc += lines_[pos_].text;
      ++pos_;
    }
    return inline_value(acc, no);
  }

  Json inline_value(const std::string& t, int no) {
    std::string s = ltrim(t);
    if (s.empty()) return Json();
    Scanner sc(s, no);
    if (s[0] == '[' || s[0] == '{' || s[0] == '"' || s[0] == '\'') {
      Json v = sc.value_flow();
      sc.ws();
      if (sc.i != s.size()) fail(no, "trailing characters after value");
      return v;
    }
    return resolve_plain(rtrim(s));
  }

  // block scalar (| or >) whose header is on line `no`; content lines are raw (comments kept)
  Json block_scalar(const std::string& header, int parent_indent, int no) {
    const bool folded = header[0] == '>';
    char chomp = 0;
    int explicit_ind = 0;
    for (size_t k = 1; k < header.size(); ++k) {
      if (header[k] == '-' || header[k] == '+') chomp = header[k];
      else if (std::isdigit(static_cast<unsigned char>(header[k]))) explicit_ind = header[k] - '0';
    }
    // raw source lines after the header line
    size_t r = static_cast<size_t>(no);  // index of next raw line (0-based)
    int ind = explicit_ind ? parent_indent + explicit_ind : -1;
    std::vector<std::string> body;
    for (; r < raw_.size(); ++r) {
      std::string ln = rtrim(raw_[r]);
      size_t li = 0;
      while (li < ln.size() && ln[li] == ' ') ++li;
      if (li == ln.size()) {
        body.push_back("");
        continue;
      }
      if (ind < 0) {
        if (static_cast<int>(li) <= parent_indent) break;
        ind = static_cast<int>(li);
      }
      if (static_cast<int>(li) < ind) break;
      body.push_back(ln.substr(static_cast<size_t>(ind)));
    }
    // drop the consumed logical lines
    while (pos_ < lines_.size() && lines_[pos_].no <= static_cast<int>(r)) ++pos_;
    size_t trailing = 0;
    while (!body.empty() && body.back().empty()) {
      body.pop_back();
      ++trailing;
    }
    std::string out;
    for (size_t k = 0; k < body.size(); ++k) {
      if (k) {
        if (folded && !body[k].empty() && !body[k - 1].empty() && body[k][0] != ' ') out += ' ';
        else out += '\n';
      }
      out += body[k];
    }
    if (chomp == '+') out += std::string(trailing + (body.empty() ? 0 : 1), '\n');
    else if (chomp != '-' && !body.empty()) out += '\n';
    return Json(out);
  }

  // value after "key:" or "- " on the same line (may be empty -> nested block / null)
  Json value_after(const std::string& rest, int line_indent, int no) {
    std::string v = ltrim(rest);
    if (!v.empty() && (v[0] == '|' || v[0] == '>')) return block_scalar(v, line_indent, no);
    if (v.empty()) {
      if (pos_ < lines_.size() && lines_[pos_].indent > line_indent) return block(lines_[pos_].indent);
      // "key:" followed by a sequence at the same indentation (compact k8s style)
      if (pos_ < lines_.size() && lines_[pos_].indent == line_indent && is_seq_item(lines_[pos_].text)) return sequence(line_indent);
      return Json();
    }
    // multi-line flow collections / quoted strings continue on deeper lines
    std::string acc = v;
    auto balanced = [](const std::string& s) {
      int depth = 0;
      bool sq = false, dq = false;
      for (size_t i = 0; i < s.size(); ++i) {
        char c = s[i];
        if (c == '\'' && !dq) sq = !sq;
        else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
        else if (!sq && !dq && (c == '[' || c == '{')) ++depth;
        else if (!sq && !dq && (c == ']' || c == '}')) --depth;
      }
      return depth <= 0 && !sq && !dq;
    };
    if (acc[0] == '[' || acc[0] == '{' || acc[0] == '"' || acc[0] == '\'') {
      while (!balanced(acc) && pos_ < lines_.size() && lines_[pos_].indent > line_indent) acc += "\n" + lines_[pos_++].text;
    } else {
      // plain multi-line scalar: every deeper line continues it (a nested block is impossible here)
      while (pos_ < lines_.size() && lines_[pos_].indent > line_indent) acc += " " + lines_[pos_++].text;
    }
    return inline_value(acc, no);
  }

  Json mapping(int indent) {
    Json out = Json::object();
    while (pos_ < lines_.size() && lines_[pos_].indent == indent) {
      const Line l = lines_[pos_];
      if (l.text == "---" || l.text == "...") break;
      size_t c = key_colon(l.text);
      if (c == std::string::npos) {
        if (is_seq_item(l.text)) break;
        fail(l.no, "expected 'key: value'");
      }
      std::string key = rtrim(l.text.substr(0, c));
      if (!key.empty() && (key[0] == '"' || key[0] == '\'')) {
        Scanner sc(key, l.no);
        key = sc.quoted();
      }
      ++pos_;
      out[key] = value_after(l.text.substr(c + 1), indent, l.no);
    }
    if (pos_ < lines_.size() && lines_[pos_].indent > indent) fail(lines_[pos_].no, "bad indentation of a mapping entry");
    return out;
  }

  Json sequence(int indent) {
    Json out = Json::array();
    while (pos_ < lines_.size() && lines_[pos_].indent == indent && is_seq_item(lines_[pos_].text)) {
      Line l = lines_[pos_];
      std::string rest = l.text.size() > 1 ? l.text.substr(2) : "";
      std::string trimmed = ltrim(rest);
      const int item_indent = indent + 2 + static_cast<int>(rest.size() - trimmed.size());
      if (trimmed.empty()) {
        ++pos_;
        out.push_back(pos_ < lines_.size() && lines_[pos_].indent > indent ? block(lines_[pos_].indent) : Json());
      } else if (is_seq_item(trimmed) || (key_colon(trimmed) != std::string::npos && trimmed[0] != '"' && trimmed[0] != '\'') ||
                 (key_colon(trimmed) != std::string::npos)) {
        // "- key: v" (or "- - x"): re-enter the block parser on a virtual line at the item indent
        lines_[pos_] = {item_indent, trimmed, l.no};
        out.push_back(block(item_indent));
      } else {
        ++pos_;
        out.push_back(value_after(trimmed, indent, l.no));
      }
    }
    return out;
  }

  const std::vector<std::string>& raw_;
  std::vector<Line> lines_;
  size_t pos_ = 0;
};

std::vector<std::vector<std::string>> split_docs(const std::string& text) {
  std::vector<std::vector<std::string>> docs(1);
  size_t st = 0;
  while (st <= text.size()) {
    size_t e = text.find('\n', st);
    std::string ln = text.substr(st, e == std::string::npos ? std::string::npos : e - st);
    std::string t = rtrim(ln);
    if (t == "---" || (t.rfind("--- ", 0) == 0)) {
      docs.emplace_back();
      if (t.size() > 4) docs.back().push_back(t.substr(4));
    } else if (t == "...") {
      docs.emplace_back();
    } else if (!(t.rfind("%", 0) == 0 && docs.back().empty())) {
      docs.back().push_back(ln);
    }
    if (e == std::string::npos) break;
    st = e + 1;
  }
  return docs;
}

bool blank_doc(const std::vector<std::string>& d) {
  for (const auto& l : d) {
    std::string t = ltrim(rtrim(strip_comment(l)));
    if (!t.empty()) return false;
  }
  return true;
}

void dump_scalar(const Json& v, std::string& out) {
  if (v.is_string()) {
    const std::string& s = v.as_string();
    Json probe = resolve_plain(s);
    bool needs = s.empty() || !probe.is_string() || s.find_first_of(":#{}[],&*!|>'\"%@`\n") != std::string::npos ||
                 s.front() == ' ' || s.back() == ' ' || s.front() == '-' || s.front() == '?';
    out += needs ? Json(s).dump() : s;
  } else {
    out += v.dump();
  }
}

void dump_node(const Json& v, int indent, std::string& out) {
  const std::string pad(static_cast<size_t>(indent), ' ');
  if (v.is_object()) {
    if (v.empty()) {
      out += "{}\n";
      return;
    }
    bool first = true;
    for (const auto& kv : v.as_object()) {
      if (!first) out += pad;
      first = false;
      dump_scalar(Json(kv.first), out);
      out += ":";
      const Json& c = kv.second;
      if ((c.is_object() || c.is_array()) && !c.empty()) {
        out += "\n" + pad + (c.is_array() ? "" : "  ");
        dump_node(c, c.is_array() ? indent : indent + 2, out);
      } else {
        out += " ";
        dump_node(c, indent + 2, out);
      }
    }
  } else if (v.is_array()) {
    if (v.empty()) {
      out += "[]\n";
      return;
    }
    bool first = true;
    for (const auto& e : v.as_array()) {
      if (!first) out += pad;
      first = false;
      out += "- ";
      dump_node(e, indent + 2, out);
    }
  } else {
    dump_scalar(v, out);
    out += "\n";
  }
}

}  // namespace

bool parse_yaml_all(const std::string& text, std::vector<Json>& docs, std::string* err) {
  docs.clear();
  try {
    for (const auto& d : split_docs(text)) {
      if (blank_doc(d)) continue;
      Parser p(d);
      docs.push_back(p.parse());
    }
    return true;
  } catch (const std::exception& e) {
    if (err) *err = e.what();
    return false;
  }
}

bool parse_yaml(const std::string& text, Json& out, std::string* err) {
  std::vector<Json> docs;
  if (!parse_yaml_all(text, docs, err)) return false;
  out = docs.empty() ? Json() : docs[0];
  return true;
}

std::string dump_yaml(const Json& v) {
  std::string out;
  dump_node(v, 0, out);
  return out;
}

}  // namespace kf
