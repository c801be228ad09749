// SPDX-License-Identifier: Apache-2.0
#include "yaml.h"

#include <cctype>
#include <cstdlib>
#include <stdexcept>

namespace pdo {
namespace yaml {

using json::Value;

namespace {

struct Line {
  int indent;
  std::string text;  // without indentation / comment
};

std::string strip_comment(const std::string& s) {
  bool sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq && (i == 0 || s[i - 1] != '\\')) dq = !dq;
    else if (c == '#' && !sq && !dq && (i == 0 || isspace((unsigned char)s[i - 1]))) return s.substr(0, i);
  }
  return s;
}

std::string rtrim(std::string s) {
  while (!s.empty() && isspace((unsigned char)s.back())) s.pop_back();
  return s;
}

std::string trim(const std::string& s) {
  size_t a = 0;
  while (a < s.size() && isspace((unsigned char)s[a])) ++a;
  return rtrim(s.substr(a));
}

Value scalar(const std::string& raw) {
  std::string s = trim(raw);
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Value();
  if (s.size() >= 2 && s.front() == '"' && s.back() == '"') {
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      if (s[i] == '\\' && i + 2 < s.size()) {
        char e = s[++i];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case '"': out.push_back('"'); break;
          case '\\': out.push_back('\\'); break;
          case '/': out.push_back('/'); break;
          default: out.push_back('\\'); out.push_back(e);
        }
      } else {
        out.push_back(s[i]);
      }
    }
    return Value(out);
  }
  if (s.size() >= 2 && s.front() == '\'' && s.back() == '\'') {
    std::string out;
    for (size_t i = 1; i + 1 < s.size(); ++i) {
      if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') ++i;
      out.push_back(s[i]);
    }
    return Value(out);
  }
  if (s == "true" || s == "True" || s == "TRUE") return Value(true);
  if (s == "false" || s == "False" || s == "FALSE") return Value(false);
  bool isint = true, isnum = true;
  size_t i = (s[0] == '-' || s[0] == '+') ? 1 : 0;
  if (i >= s.size()) isint = isnum = false;
  int dots = 0, exps = 0;
  for (size_t j = i; j < s.size(); ++j) {
    char c = s[j];
    if (isdigit((unsigned char)c)) continue;
    isint = false;
    if (c == '.') ++dots;
    else if ((c == 'e' || c == 'E') && j > i) ++exps;
    else if ((c == '-' || c == '+') && j > 0 && (s[j - 1] == 'e' || s[j - 1] == 'E')) continue;
    else isnum = false;
  }
  if (isint && s.size() - i < 19) return Value((int64_t)strtoll(s.c_str(), nullptr, 10));
  if (isnum && dots <= 1 && exps <= 1 && (dots || exps)) return Value(strtod(s.c_str(), nullptr));
  return Value(s);
}

// split a flow collection body at top-level commas
std::vector<std::string> split_flow(const std::string& body) {
  std::vector<std::string> out;
  int depth = 0;
  bool sq = false, dq = false;
  std::string cur;
  for (char c : body) {
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    if (!sq && !dq) {
      if (c == '[' || c == '{') ++depth;
      else if (c == ']' || c == '}') --depth;
      else if (c == ',' && depth == 0) {
        out.push_back(trim(cur));
        cur.clear();
        continue;
      }
    }
    cur.push_back(c);
  }
  if (!trim(cur).empty()) out.push_back(trim(cur));
  return out;
}

// find the ':' that separates key and value (outside quotes/brackets)
size_t key_colon(const std::string& s) {
  bool sq = false, dq = false;
  int depth = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '\'' && !dq) sq = !sq;
    else if (c == '"' && !sq) dq = !dq;
    else if (!sq && !dq) {
      if (c == '[' || c == '{') ++depth;
      else if (c == ']' || c == '}') --depth;
      else if (c == ':' && depth == 0 && (i + 1 == s.size() || s[i + 1] == ' ' || s[i + 1] == '\t')) return i;
    }
  }
  return std::string::npos;
}

Value flow(const std::string& s) {
  std::string t = trim(s);
  if (t.size() >= 2 && t.front() == '[' && t.back() == ']') {
    Value a = Value::array();
    for (auto& it : split_flow(t.substr(1, t.size() - 2))) a.push_back(flow(it));
    return a;
  }
  if (t.size() >= 2 && t.front() == '{' && t.back() == '}') {
    Value o = Value::object();
    for (auto& it : split_flow(t.substr(1, t.size() - 2))) {
      size_t c = key_colon(it);
      if (c == std::string::npos) {
        o[scalar(it).str(it)] = Value();
        continue;
      }
      o[scalar(it.substr(0, c)).str(trim(it.substr(0, c)))] = flow(it.substr(c + 1));
    }
    return o;
  }
  return scalar(t);
}

struct Parser {
  std::vector<Line> lines;
  size_t i = 0;

  bool is_seq(const Line& l) const { return l.text == "-" || l.text.rfind("- ", 0) == 0; }

  Value node(int indent) {
    if (i >= lines.size()) return Value();
    const Line& l = lines[i];
    if (l.indent < indent) return Value();
    if (is_seq(l)) return seq(l.indent);
    if (key_colon(l.text) != std::string::npos) return map(l.indent);
    // plain (possibly multi-line) scalar
    std::string s = l.text;
    ++i;
    while (i < lines.size() && lines[i].indent > indent && !is_seq(lines[i]) &&
           key_colon(lines[i].text) == std::string::npos) {
      s += " " + lines[i].text;
      ++i;
    }
    return flow(s);
  }

  Value block_scalar(int parent_indent, const std::string& style) {
    const bool literal = style[0] == '|';
    const bool keep = style.find('+') != std::string::npos;
    const bool strip = style.find('-') != std::string::npos;
    std::string out;
    int bi = -1;
    while (i < lines.size() && (lines[i].indent > parent_indent || lines[i].text.empty())) {
      if (bi < 0) bi = lines[i].indent;
      std::string pad(lines[i].indent > bi ? lines[i].indent - bi : 0, ' ');
      std::string t = pad + lines[i].text;
      if (literal) out += t + "\n";
      else out += (out.empty() || out.back() == '\n' ? "" : " ") + t;
      ++i;
    }
    if (!literal) out += "\n";
    if (strip) {
      while (!out.empty() && out.back() == '\n') out.pop_back();
    } else if (!keep) {
      while (out.size() >= 2 && out[out.size() - 1] == '\n' && out[out.size() - 2] == '\n') out.pop_back();
    }
    return Value(out);
  }

  Value value_after_key(int indent, const std::string& rest) {
    std::string v = trim(rest);
    if (!v.empty() && (v[0] == '|' || v[0] == '>')) return block_scalar(indent, v);
    if (!v.empty()) return flow(v);
    if (i >= lines.size()) return Value();
    if (lines[i].indent > indent) return node(lines[i].indent);
    if (lines[i].indent == indent && is_seq(lines[i])) return seq(indent);  // "key:\n- a"
    return Value();
  }

  Value map(int indent) {
    Value o = Value::object();
    while (i < lines.size() && lines[i].indent == indent && !is_seq(lines[i])) {
      const std::string t = lines[i].text;
      size_t c = key_colon(t);
      if (c == std::string::npos) throw std::runtime_error("yaml: expected 'key: value' near: " + t);
      std::string key = scalar(t.substr(0, c)).str(trim(t.substr(0, c)));
      ++i;
      o[key] = value_after_key(indent, t.substr(c + 1));
    }
    return o;
  }

  Value seq(int indent) {
    Value a = Value::array();
    while (i < lines.size() && lines[i].indent == indent && is_seq(lines[i])) {
      std::string rest = lines[i].text.size() > 1 ? lines[i].text.substr(2) : "";
      size_t lead = 0;
      while (lead < rest.size() && rest[lead] == ' ') ++lead;
      rest = rest.substr(lead);
      if (trim(rest).empty()) {
        ++i;
        a.push_back(i < lines.size() && lines[i].indent > indent ? node(lines[i].indent) : Value());
        continue;
      }
      // rewrite "- x" as a line indented past the dash and parse it as a node
      lines[i].indent = indent + 2 + (int)lead;
      lines[i].text = rest;
      a.push_back(node(lines[i].indent));
    }
    return a;
  }
};

}  // namespace

std::vector<Value> parse_all(const std::string& text) {
  std::vector<Value> docs;
  std::vector<Line> cur;
  auto flush = [&]() {
    bool any = false;
    for (auto& l : cur)
      if (!l.text.empty()) any = true;
    if (any) {
      Parser p;
      for (auto& l : cur)
        if (!l.text.empty()) p.lines.push_back(l);
      docs.push_back(p.node(p.lines.empty() ? 0 : p.lines[0].indent));
    }
    cur.clear();
  };
  size_t pos = 0;
  bool in_block = false;
  int block_indent = 0;
  while (pos <= text.size()) {
    size_t nl = text.find('\n', pos);
    std::string raw = text.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
    if (!raw.empty() && raw.back() == '\r') raw.pop_back();
    int ind = 0;
    while (ind < (int)raw.size() && raw[ind] == ' ') ++ind;
    if (raw.rfind("---", 0) == 0 && !in_block) {
      flush();
    } else if (raw == "...") {
      flush();
    } else {
      std::string body = in_block && ind > block_indent ? raw.substr(ind) : rtrim(strip_comment(raw.substr(ind)));
      if (in_block && ind <= block_indent && !trim(raw).empty()) in_block = false;
      if (!in_block) body = rtrim(strip_comment(raw.substr(std::min((size_t)ind, raw.size()))));
      if (in_block && trim(raw).empty()) cur.push_back(Line{block_indent + 1, ""});
      else if (!trim(body).empty() || in_block) cur.push_back(Line{ind, body});
      // detect the start of a literal/folded block scalar
      if (!in_block) {
        std::string t = trim(body);
        if (!t.empty() && (t.back() == '|' || t.back() == '>' ||
                           (t.size() >= 2 && (t[t.size() - 2] == '|' || t[t.size() - 2] == '>') &&
                            (t.back() == '-' || t.back() == '+')))) {
          size_t c = key_colon(t);
          std::string v = c == std::string::npos ? t : trim(t.substr(c + 1));
          if (!v.empty() && (v[0] == '|' || v[0] == '>')) {
            in_block = true;
            block_indent = ind;
          }
        }
      }
    }
    if (nl == std::string::npos) break;
    pos = nl + 1;
  }
  flush();
  return docs;
}

Value parse(const std::string& text) {
  auto d = parse_all(text);
  return d.empty() ? Value() : d[0];
}

}  // namespace yaml
}  // namespace pdo
