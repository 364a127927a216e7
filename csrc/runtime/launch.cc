// gst-launch description parser (the grammar the reference's tooling
// documents in tools/development/parser/grammar.y): chains of elements with
// `prop=value` settings joined by `!`, inline caps filters, named references
// `name.` / `name.pad`, several chains separated by whitespace.
#include <cctype>

#include "core/log.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

struct Endpoint {
  int elem = -1;          // index into elems (when an element literal)
  std::string ref;        // referenced element name
  std::string pad;        // pad name hint
};

struct ElemDecl {
  std::string factory;
  std::vector<std::pair<std::string, std::string>> props;
  std::string name;
};

struct LinkDecl {
  Endpoint src, sink;
  std::string caps;
};

class Lexer {
 public:
  explicit Lexer(const std::string& s) : s_(s) {}
  void ws() {
    while (p_ < s_.size() && std::isspace(static_cast<unsigned char>(s_[p_]))) ++p_;
  }
  bool eof() {
    ws();
    return p_ >= s_.size();
  }
  char peek() {
    ws();
    return p_ < s_.size() ? s_[p_] : '\0';
  }
  bool eat(char c) {
    ws();
    if (p_ < s_.size() && s_[p_] == c) {
      ++p_;
      return true;
    }
    return false;
  }
  // a raw word: until whitespace or '!' ; quoted sections and bracket nesting kept
  std::string word() {
    ws();
    std::string r;
    int depth = 0;
    while (p_ < s_.size()) {
      char c = s_[p_];
      if (c == '"' || c == '\'') {
        char q = c;
        r += c;
        ++p_;
        while (p_ < s_.size() && s_[p_] != q) {
          if (s_[p_] == '\\' && p_ + 1 < s_.size()) r += s_[p_++];
          r += s_[p_++];
        }
        if (p_ < s_.size()) r += s_[p_++];
        continue;
      }
      if (c == '{' || c == '[' || c == '(' || c == '<') ++depth;
      if (c == '}' || c == ']' || c == ')' || c == '>') --depth;
      if (depth <= 0 && (std::isspace(static_cast<unsigned char>(c)) || c == '!')) break;
      r += c;
      ++p_;
    }
    return r;
  }
  // caps: mime followed by ", field=value" groups (spaces allowed around commas)
  std::string caps() {
    std::string r = word();
    while (true) {
      size_t save = p_;
      ws();
      if (p_ < s_.size() && s_[p_] == ',') {
        ++p_;
        std::string w = word();
        r += "," + w;
        continue;
      }
      if (!r.empty() && r.back() == ',') {
        std::string w = word();
        r += w;
        continue;
      }
      p_ = save;
      break;
    }
    return r;
  }
  size_t pos() const { return p_; }
  void set_pos(size_t p) { p_ = p; }

 private:
  const std::string& s_;
  size_t p_ = 0;
};

std::string unquote(const std::string& v) {
  if (v.size() >= 2 && ((v.front() == '"' && v.back() == '"') || (v.front() == '\'' && v.back() == '\''))) {
    std::string r;
    for (size_t i = 1; i + 1 < v.size(); ++i) {
      if (v[i] == '\\' && i + 2 < v.size()) {
        r += v[++i];
        continue;
      }
      r += v[i];
    }
    return r;
  }
  return v;
}

bool looks_like_caps(const std::string& w) {
  // mime type "type/subtype" before any ',' or '(' and without '='
  size_t end = w.find_first_of(",(");
  std::string head = w.substr(0, end);
  if (head.find('=') != std::string::npos) return false;
  size_t slash = head.find('/');
  return slash != std::string::npos && slash > 0 && slash + 1 < head.size() && head.find('.') == std::string::npos;
}

bool looks_like_ref(const std::string& w) {
  if (w.find('=') != std::string::npos || w.find('/') != std::string::npos) return false;
  size_t dot = w.find('.');
  return dot != std::string::npos && dot > 0;
}

}  // namespace

std::unique_ptr<Pipeline> parse_launch(const std::string& description) {
  ensure_builtin_elements();
  Lexer lx(description);
  std::vector<ElemDecl> elems;
  std::vector<LinkDecl> links;

  bool have_prev = false;
  Endpoint prev;
  bool pending_link = false;  // saw '!'
  std::string pending_caps;

  auto connect = [&](const Endpoint& cur) {
    if (pending_link) {
      if (!have_prev) throw Error("syntax error: link without source near position " + std::to_string(lx.pos()));
      links.push_back(LinkDecl{prev, cur, pending_caps});
      pending_caps.clear();
      pending_link = false;
    }
    prev = cur;
    have_prev = true;
  };

  while (!lx.eof()) {
    if (lx.eat('!')) {
      if (pending_link) throw Error("syntax error: '! !'");
      pending_link = true;
      continue;
    }
    size_t save = lx.pos();
    std::string w = lx.word();
    if (w.empty()) throw Error("syntax error at position " + std::to_string(lx.pos()));
    if (looks_like_caps(w)) {
      lx.set_pos(save);
      std::string c = lx.caps();
      if (!pending_link) throw Error("syntax error: caps '" + c + "' must follow '!'");
      if (!have_prev) throw Error("syntax error: caps without source");
      // implicit capsfilter element
      ElemDecl d;
      d.factory = "capsfilter";
      d.props.emplace_back("caps", unquote(c));
      elems.push_back(d);
      Endpoint ep;
      ep.elem = static_cast<int>(elems.size()) - 1;
      connect(ep);
      continue;
    }
    if (looks_like_ref(w)) {
      Endpoint ep;
      size_t dot = w.find('.');
      ep.ref = w.substr(0, dot);
      ep.pad = w.substr(dot + 1);
      if (!pending_link) {
        // starts a new chain
        prev = ep;
        have_prev = true;
      } else {
        connect(ep);
      }
      continue;
    }
    if (w.find('=') != std::string::npos) throw Error("syntax error: property '" + w + "' without element");
    // element literal
    ElemDecl d;
    d.factory = w;
    while (!lx.eof()) {
      size_t s2 = lx.pos();
      char c = lx.peek();
      if (c == '!') break;
      std::string pw = lx.word();
      auto eq = pw.find('=');
      if (eq == std::string::npos || looks_like_caps(pw)) {
        lx.set_pos(s2);
        break;
      }
      std::string key = strip(pw.substr(0, eq));
      std::string val = strip(pw.substr(eq + 1));
      if (val.empty()) {
        // `key= value` form
        size_t s3 = lx.pos();
        if (!lx.eof() && lx.peek() != '!') {
          val = lx.word();
        } else {
          lx.set_pos(s3);
        }
      }
      val = unquote(val);
      if (key == "name")
        d.name = val;
      else
        d.props.emplace_back(key, val);
    }
    elems.push_back(d);
    Endpoint ep;
    ep.elem = static_cast<int>(elems.size()) - 1;
    if (!pending_link && have_prev) {
      // whitespace-separated new chain
      have_prev = false;
    }
    connect(ep);
  }
  if (pending_link) throw Error("syntax error: trailing '!'");

  auto pipe = std::make_unique<Pipeline>();
  std::vector<Element*> made;
  for (const auto& d : elems) {
    std::unique_ptr<Element> e = make_element(d.factory, d.name);
    if (!d.name.empty()) e->set_name(d.name);
    for (const auto& kv : d.props) {
      try {
        e->set_property(kv.first, kv.second);
      } catch (const std::exception& ex) {
        throw Error(strfmt("could not set property \"", kv.first, "\" in element \"", d.factory, "\" to \"",
                           kv.second, "\": ", ex.what()));
      }
    }
    made.push_back(pipe->add(std::move(e)));
  }
  auto resolve = [&](const Endpoint& ep) -> Element* {
    if (ep.elem >= 0) return made[ep.elem];
    Element* e = pipe->get_by_name(ep.ref);
    if (!e) throw Error("no element named \"" + ep.ref + "\"");
    return e;
  };
  for (const auto& l : links) {
    Element* a = resolve(l.src);
    Element* b = resolve(l.sink);
    if (!pipe->link(a, l.src.pad, b, l.sink.pad, l.caps))
      throw Error(strfmt("could not link ", a->name(), l.src.pad.empty() ? "" : "." + l.src.pad, " to ", b->name(),
                         l.sink.pad.empty() ? "" : "." + l.sink.pad));
  }
  return pipe;
}

}  // namespace nnsx
