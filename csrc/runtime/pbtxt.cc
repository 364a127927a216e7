// Pipeline <-> MediaPipe-style pbtxt graph text.
//
// Reference: tools/development/parser/convert.c (gst-launch -> pbtxt; node
// names `<factory>` / `<factory>_<n>`, internal streams
// `<factory>_<index>_<srcpad>`, sources / sinks become the graph's
// input_stream / output_stream) and toplevel.c:108-111, where the reverse
// direction is "NYI".  nnsx converts both ways.  Caps filters are link
// attributes in gst-launch syntax, so capsfilter elements are bridged over
// (with_options keeps them as `caps` node options of their consumer).
#include "runtime/pbtxt.h"

#include <cctype>
#include <cstring>
#include <map>
#include <regex>
#include <set>
#include <sstream>

#include <algorithm>

#include "core/util.h"

namespace nnsx {

namespace {

bool is_capsfilter(const Element* e) { return e->factory() == "capsfilter"; }

// downstream consumer pad of `src`, skipping capsfilters (caps collected)
Pad* downstream(Pad* src, std::string* caps) {
  Pad* p = src ? src->peer() : nullptr;
  while (p && is_capsfilter(p->parent())) {
    if (caps) *caps = p->parent()->get_property("caps");
    auto outs = p->parent()->src_pads();
    p = outs.empty() ? nullptr : outs[0]->peer();
  }
  return p;
}

// upstream producer pad of `sink`, skipping capsfilters
Pad* upstream(Pad* sink, std::string* caps) {
  Pad* p = sink ? sink->peer() : nullptr;
  while (p && is_capsfilter(p->parent())) {
    if (caps) *caps = p->parent()->get_property("caps");
    auto ins = p->parent()->sink_pads();
    p = ins.empty() ? nullptr : ins[0]->peer();
  }
  return p;
}

std::string quote(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o.push_back('\\');
    o.push_back(c);
  }
  return o + "\"";
}

}  // namespace

std::string pipeline_to_pbtxt(const Pipeline& pipeline, bool with_options) {
  std::vector<Element*> elems;
  for (Element* e : pipeline.elements())
    if (!is_capsfilter(e)) elems.push_back(e);
  std::map<std::string, int> seen;
  std::map<const Element*, int> index;
  for (Element* e : elems) index[e] = seen[e->factory()]++;
  auto node_name = [&](const Element* e) {
    const int i = index.at(e);
    return i == 0 ? e->factory() : strfmt(e->factory(), "_", i + 1);
  };
  auto linked_src = [](const Element* e) {
    std::vector<Pad*> v;
    for (Pad* p : e->src_pads())
      if (downstream(p, nullptr)) v.push_back(p);
    return v;
  };
  auto linked_sink = [](const Element* e) {
    std::vector<Pad*> v;
    for (Pad* p : e->sink_pads())
      if (upstream(p, nullptr)) v.push_back(p);
    return v;
  };
  auto pad_index = [&](const Element* e, const Pad* p) {
    auto v = linked_src(e);
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i] == p) return static_cast<int>(i);
    return 0;
  };
  // properties that differ from a fresh element of the same factory
  auto changed = [](const Element* e) {
    std::vector<std::string> opts;
    auto fresh = make_element(e->factory(), "");
    for (auto& ps : e->properties()) {
      if (!ps.writable || ps.name == "name" || !ps.get) continue;
      try {
        const std::string v = ps.get();
        if (v != fresh->get_property(ps.name)) opts.push_back(ps.name + "=" + v);
      } catch (...) {
      }
    }
    return opts;
  };
  std::ostringstream os;
  std::vector<std::pair<std::string, std::vector<std::string>>> io_opts;
  for (Element* e : elems) {
    const bool in = linked_sink(e).empty(), out = linked_src(e).empty();
    if (in) os << "input_stream: " << quote(node_name(e)) << "\n";
    if (out) os << "output_stream: " << quote(node_name(e)) << "\n";
    if (with_options && (in || out)) {
      auto o = changed(e);
      if (!o.empty()) io_opts.emplace_back(node_name(e), o);
    }
  }
  // nnsx extension: properties of the graph's sources / sinks
  for (auto& io : io_opts) {
    os << "stream_options: {\n\tstream: " << quote(io.first) << "\n";
    for (auto& o : io.second) os << "\toption: " << quote(o) << "\n";
    os << "}\n";
  }
  for (Element* e : elems) {
    auto ins = linked_sink(e), outs = linked_src(e);
    if (ins.empty() || outs.empty()) continue;
    os << "\nnode: {\n\tcalculator: " << quote(e->factory() + "Calculator") << "\n";
    std::vector<std::string> caps_in;
    for (Pad* sp : ins) {
      std::string caps;
      Pad* up = upstream(sp, &caps);
      if (!caps.empty()) caps_in.push_back(caps);
      const Element* u = up->parent();
      os << "\tinput_stream: "
         << quote(linked_sink(u).empty() ? node_name(u) : strfmt(u->factory(), "_", index.at(u), "_", pad_index(u, up)))
         << "\n";
    }
    for (Pad* sp : outs) {
      const Element* d = downstream(sp, nullptr)->parent();
      os << "\toutput_stream: "
         << quote(linked_src(d).empty() ? node_name(d) : strfmt(e->factory(), "_", index.at(e), "_", pad_index(e, sp)))
         << "\n";
    }
    if (with_options) {
      std::vector<std::string> opts = changed(e);
      for (auto& c : caps_in) opts.push_back("caps=" + c);
      if (!opts.empty()) {
        os << "\tnode_options: {\n";
        for (auto& o : opts) os << "\t\toption: " << quote(o) << "\n";
        os << "\t}\n";
      }
    }
    os << "}\n";
  }
  return os.str();
}

std::string pbtxt_to_launch(const std::string& text, std::string* err) {
  struct Node {
    std::string factory, name;
    std::vector<std::string> ins, outs, opts;
  };
  std::vector<std::string> graph_in, graph_out;
  std::vector<Node> nodes;
  std::map<std::string, std::vector<std::string>> stream_opts;
  // tokenizer: identifiers, quoted strings, { } :
  std::vector<std::string> tok;
  std::vector<bool> is_str;
  for (size_t i = 0; i < text.size();) {
    const char c = text[i];
    if (std::isspace(static_cast<unsigned char>(c))) {
      ++i;
    } else if (c == '#') {
      while (i < text.size() && text[i] != '\n') ++i;
    } else if (c == '"') {
      std::string s;
      for (++i; i < text.size() && text[i] != '"'; ++i) {
        if (text[i] == '\\' && i + 1 < text.size()) ++i;
        s.push_back(text[i]);
      }
      ++i;
      tok.push_back(s);
      is_str.push_back(true);
    } else if (c == '{' || c == '}' || c == ':' || c == '[' || c == ']') {
      tok.emplace_back(1, c);
      is_str.push_back(false);
      ++i;
    } else {
      std::string s;
      while (i < text.size() && !std::isspace(static_cast<unsigned char>(text[i])) && !std::strchr("{}:\"[]#", text[i]))
        s.push_back(text[i++]);
      tok.push_back(s);
      is_str.push_back(false);
    }
  }
  auto fail = [&](const std::string& m) {
    if (err) *err = "pbtxt: " + m;
    return std::string();
  };
  size_t i = 0;
  auto expect_value = [&](std::string* v) {
    if (i < tok.size() && tok[i] == ":" && !is_str[i]) ++i;
    if (i >= tok.size() || !is_str[i]) return false;
    *v = tok[i++];
    return true;
  };
  while (i < tok.size()) {
    const std::string key = tok[i++];
    if (key == "input_stream" || key == "output_stream") {
      std::string v;
      if (!expect_value(&v)) return fail("expected a string after " + key);
      (key == "input_stream" ? graph_in : graph_out).push_back(v);
    } else if (key == "node") {
      if (i < tok.size() && tok[i] == ":") ++i;
      if (i >= tok.size() || tok[i] != "{") return fail("expected '{' after node");
      ++i;
      Node n;
      int depth = 1;
      while (i < tok.size() && depth > 0) {
        const std::string k = tok[i++];
        if (k == "}") {
          --depth;
        } else if (k == "{") {
          ++depth;
        } else if (k == "calculator" || k == "input_stream" || k == "output_stream" || k == "option") {
          std::string v;
          if (!expect_value(&v)) return fail("expected a string after " + k);
          if (k == "calculator") {
            n.factory = v.size() > 10 && v.compare(v.size() - 10, 10, "Calculator") == 0 ? v.substr(0, v.size() - 10) : v;
          } else if (k == "input_stream") {
            n.ins.push_back(v);
          } else if (k == "output_stream") {
            n.outs.push_back(v);
          } else {
            n.opts.push_back(v);
          }
        }
      }
      if (n.factory.empty()) return fail("node without a calculator");
      nodes.push_back(n);
    } else if (key == "stream_options") {
      if (i < tok.size() && tok[i] == ":") ++i;
      if (i >= tok.size() || tok[i] != "{") return fail("expected '{' after stream_options");
      ++i;
      std::string stream;
      std::vector<std::string> opts;
      while (i < tok.size() && tok[i] != "}") {
        const std::string k = tok[i++];
        std::string v;
        if ((k == "stream" || k == "option") && !expect_value(&v)) return fail("expected a string after " + k);
        if (k == "stream") stream = v;
        if (k == "option") opts.push_back(v);
      }
      ++i;
      stream_opts[stream] = opts;
    } else if (key == ":" || key == "}" || key == "{") {
      continue;
    } else {
      // unknown top-level field: skip its value / block
      if (i < tok.size() && tok[i] == ":") ++i;
      if (i < tok.size() && tok[i] == "{") {
        int depth = 0;
        do {
          if (tok[i] == "{") ++depth;
          if (tok[i] == "}") --depth;
          ++i;
        } while (i < tok.size() && depth > 0);
      } else if (i < tok.size()) {
        ++i;
      }
    }
  }
  // graph streams name their elements: "<factory>" or "<factory>_<n>"
  static const std::regex suffix("^(.*)_[0-9]+$");
  auto factory_of = [&](const std::string& s) {
    std::smatch m;
    if (element_exists(s)) return s;
    if (std::regex_match(s, m, suffix) && element_exists(m[1].str())) return m[1].str();
    return s;
  };
  auto ident = [](std::string s) {
    for (auto& c : s)
      if (!std::isalnum(static_cast<unsigned char>(c)) && c != '_' && c != '-') c = '_';
    return s;
  };
  std::ostringstream os;
  auto props = [&](const std::vector<std::string>& opts) {
    for (auto& o : opts) {
      const size_t eq = o.find('=');
      os << " " << (eq == std::string::npos ? o : o.substr(0, eq) + "=" + quote(o.substr(eq + 1)));
    }
  };
  std::map<std::string, std::string> producer;  // stream -> element name
  for (auto& s : graph_in) {
    os << factory_of(s) << " name=" << ident(s);
    props(stream_opts[s]);
    os << " ";
    producer[s] = ident(s);
  }
  std::map<std::string, int> seen;
  for (auto& n : nodes) {
    const int k = seen[n.factory]++;
    n.name = ident(k == 0 ? "n_" + n.factory : strfmt("n_", n.factory, "_", k + 1));
    os << n.factory << " name=" << n.name;
    std::string caps;
    std::vector<std::string> rest;
    for (auto& o : n.opts) {
      if (o.compare(0, 5, "caps=") == 0)
        caps = o.substr(5);
      else
        rest.push_back(o);
    }
    props(rest);
    os << " ";
    n.opts.assign(1, caps);  // remember the input caps for the links below
    for (auto& s : n.outs) producer[s] = n.name;
  }
  std::set<std::string> sinks_done;
  for (auto& s : graph_out) {
    if (producer.count(s) && std::find(graph_in.begin(), graph_in.end(), s) != graph_in.end()) continue;
    os << factory_of(s) << " name=" << ident(s);
    props(stream_opts[s]);
    os << " ";
  }
  // links: every node input / graph output consumes the stream's producer
  auto link = [&](const std::string& stream, const std::string& consumer, const std::string& caps) {
    auto it = producer.find(stream);
    if (it == producer.end()) return false;
    os << it->second << ". ! " << (caps.empty() ? "" : caps + " ! ") << consumer << ". ";
    return true;
  };
  for (auto& n : nodes)
    for (auto& s : n.ins)
      if (!link(s, n.name, n.opts[0])) return fail("no producer for stream " + s);
  for (auto& s : graph_out) {
    // a graph output is fed by the node that names it as an output stream
    bool ok = false;
    for (auto& n : nodes)
      for (auto& o : n.outs)
        if (o == s && !ok) ok = link(s, ident(s), std::string());
    if (!ok) return fail("no producer for output stream " + s);
  }
  std::string out = os.str();
  while (!out.empty() && out.back() == ' ') out.pop_back();
  return out;
}

}  // namespace nnsx
