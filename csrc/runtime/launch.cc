// gst-launch description parser (the grammar the reference's tooling
// documents in tools/development/parser/grammar.y): chains of elements with
// `prop=value` settings joined by `!`, inline caps filters, named references
// `name.` / `name.pad`, several chains separated by whitespace, and bins
// `( ... )` / `<type>.( ... )` (flattened into the pipeline).
#include <cctype>
#include <cstring>

#include "core/log.h"
#include "runtime/pipeline.h"

namespace nnsx {

namespace {

struct Endpoint {
  int elem = -1;          // index into elems (when an element literal)
  int group = -1;         // index into groups (a bin)
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
      if (c == ')' && depth == 0) break;  // closes a bin
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
  // [A-Za-z0-9_-]* at the cursor (after whitespace)
  std::string ident() {
    ws();
    std::string r;
    while (p_ < s_.size() && (std::isalnum(static_cast<unsigned char>(s_[p_])) || s_[p_] == '_' || s_[p_] == '-'))
      r += s_[p_++];
    return r;
  }
  // exactly `t` at the cursor, no whitespace skipped
  bool raw_eat(const char* t) {
    const size_t n = std::strlen(t);
    if (s_.compare(p_, n, t) != 0) return false;
    p_ += n;
    return true;
  }

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

// One chain list: chains of elements / caps / references joined by '!',
// separated by whitespace; `( ... )` and `<type>.( ... )` open a bin whose
// leading `prop=value`s (name=) belong to the bin.  nnsx flattens bins into the
// pipeline: a bin links like its first element (as a link's sink) and its last
// element (as a link's source) -- the pads gst-launch would ghost
// (tools/development/parser/grammar.y: bin rules, gst_parse_perform_link).
struct Group {
  int head = -1, tail = -1;
  std::string name;
};

class LaunchParser {
 public:
  explicit LaunchParser(const std::string& d) : lx_(d) {}
  std::vector<ElemDecl> elems;
  std::vector<LinkDecl> links;
  std::vector<Group> groups;

  // parses until ')' (in a bin) or the end; returns the group it filled
  Group parse_list(bool in_bin) {
    Group g;
    bool have_prev = false;
    Endpoint prev;
    bool pending_link = false;  // saw '!'
    std::string pending_caps;
    bool bin_props = in_bin;    // a bin's own name= comes before its first element

    auto note = [&](const Endpoint& ep) {
      const int e = ep.group >= 0 ? groups[ep.group].tail : ep.elem;
      const int h = ep.group >= 0 ? groups[ep.group].head : ep.elem;
      if (g.head < 0 && h >= 0) g.head = h;
      if (e >= 0) g.tail = e;
    };
    auto connect = [&](const Endpoint& cur) {
      if (pending_link) {
        if (!have_prev) throw Error("syntax error: link without source near position " + std::to_string(lx_.pos()));
        links.push_back(LinkDecl{prev, cur, pending_caps});
        pending_caps.clear();
        pending_link = false;
      }
      prev = cur;
      have_prev = true;
      note(cur);
    };

    while (!lx_.eof()) {
      if (lx_.peek() == ')') {
        if (!in_bin) throw Error("syntax error: unbalanced ')'");
        lx_.eat(')');
        if (pending_link) throw Error("syntax error: trailing '!' in a bin");
        return g;
      }
      if (lx_.eat('!')) {
        if (pending_link) throw Error("syntax error: '! !'");
        pending_link = true;
        continue;
      }
      if (open_bin()) {
        const int gi = static_cast<int>(groups.size());
        groups.emplace_back();
        Group inner = parse_list(true);
        groups[gi] = inner;
        if (inner.head < 0) throw Error("syntax error: empty bin");
        Endpoint ep;
        ep.group = gi;
        if (!pending_link && have_prev) have_prev = false;  // a new chain
        connect(ep);
        bin_props = false;
        continue;
      }
      size_t save = lx_.pos();
      std::string w = lx_.word();
      if (w.empty()) throw Error("syntax error at position " + std::to_string(lx_.pos()));
      if (bin_props && w.find('=') != std::string::npos && !looks_like_caps(w)) {
        auto eq = w.find('=');
        const std::string key = strip(w.substr(0, eq)), val = unquote(strip(w.substr(eq + 1)));
        if (key == "name")
          g.name = val;
        else
          NNSX_LOGW("launch", "bin property ", key, " ignored (bins are flattened)");
        continue;
      }
      bin_props = false;
      if (looks_like_caps(w)) {
        lx_.set_pos(save);
        std::string c = lx_.caps();
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
      while (!lx_.eof()) {
        size_t s2 = lx_.pos();
        char c = lx_.peek();
        if (c == '!' || c == ')' || c == '(') break;
        if (open_bin()) {  // `<type>.(` starts a bin, not a property
          lx_.set_pos(s2);
          break;
        }
        std::string pw = lx_.word();
        auto eq = pw.find('=');
        if (eq == std::string::npos || looks_like_caps(pw)) {
          lx_.set_pos(s2);
          break;
        }
        std::string key = strip(pw.substr(0, eq));
        std::string val = strip(pw.substr(eq + 1));
        if (val.empty()) {
          // `key= value` form
          size_t s3 = lx_.pos();
          if (!lx_.eof() && lx_.peek() != '!') {
            val = lx_.word();
          } else {
            lx_.set_pos(s3);
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
    if (in_bin) throw Error("syntax error: unterminated bin '('");
    if (pending_link) throw Error("syntax error: trailing '!'");
    return g;
  }

 private:
  // '(' or '<bintype>.(' at the cursor: consumed, true
  bool open_bin() {
    const size_t save = lx_.pos();
    if (lx_.eat('(')) return true;
    std::string id = lx_.ident();
    if (!id.empty() && lx_.raw_eat(".(")) return true;
    lx_.set_pos(save);
    return false;
  }
  Lexer lx_;
};

std::unique_ptr<Pipeline> parse_launch(const std::string& description) {
  ensure_builtin_elements();
  LaunchParser ps(description);
  ps.parse_list(false);
  std::vector<ElemDecl>& elems = ps.elems;
  std::vector<LinkDecl>& links = ps.links;
  std::vector<Group>& groups = ps.groups;

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
  // element, bin (as a link's source: its last element; as a sink: its first)
  // or a named reference (an element, else a named bin)
  auto resolve = [&](const Endpoint& ep, bool as_src) -> Element* {
    if (ep.elem >= 0) return made[ep.elem];
    if (ep.group >= 0) return made[as_src ? groups[ep.group].tail : groups[ep.group].head];
    Element* e = pipe->get_by_name(ep.ref);
    if (e) return e;
    for (const auto& g : groups)
      if (g.name == ep.ref) return made[as_src ? g.tail : g.head];
    throw Error("no element named \"" + ep.ref + "\"");
  };
  for (const auto& l : links) {
    Element* a = resolve(l.src, true);
    Element* b = resolve(l.sink, false);
    if (!pipe->link(a, l.src.pad, b, l.sink.pad, l.caps))
      throw Error(strfmt("could not link ", a->name(), l.src.pad.empty() ? "" : "." + l.src.pad, " to ", b->name(),
                         l.sink.pad.empty() ? "" : "." + l.sink.pad));
  }
  return pipe;
}

}  // namespace nnsx
