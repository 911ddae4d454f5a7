// config.h — `key: value` configuration (reference: utils/ConfigParser.h:25-129).
//
// Syntax and semantics preserved from the reference:
//   * one `key: value` per line, split on the FIRST ':' (so values may contain
//     ':' — e.g. `listen_addr: tcp://127.0.0.1:8080`);
//   * lines starting with '#' are comments, blank lines ignored;
//   * `import <path>` recursively parses another file;
//   * FIRST definition wins (std::map::insert, ConfigParser.h:112-119) — so a
//     file can `import` shared defaults AFTER its own overrides;
//   * `get_config` on a missing key is an error (CHECK in the reference).
// Additions: relative imports resolve against the importing file, import
// cycles are detected, `set` overrides, `register_config` provides defaults
// (the reference's is commented out, ConfigParser.h:61-66, yet used by its
// tests), and values may come from strings (Python-side configs / CLI).
#pragma once
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "common.h"
#include "string_util.h"

namespace ss {

class ConfigParser {
 public:
  struct Item {
    std::string value;
    Item() = default;
    explicit Item(std::string v) : value(std::move(v)) {}
    int to_int32() const {
      SS_CHECK_MSG(!value.empty(), "empty config value");
      return std::stoi(value);
    }
    long long to_int64() const {
      SS_CHECK_MSG(!value.empty(), "empty config value");
      return std::stoll(value);
    }
    float to_float() const {
      SS_CHECK_MSG(!value.empty(), "empty config value");
      return std::stof(value);
    }
    double to_double() const {
      SS_CHECK_MSG(!value.empty(), "empty config value");
      return std::stod(value);
    }
    const std::string& to_string() const { return value; }
    bool to_bool() const {
      SS_CHECK_MSG(value == "true" || value == "false",
                   "bool config must be 'true' or 'false', got '" << value << "'");
      return value == "true";
    }
  };

  ConfigParser() = default;
  explicit ConfigParser(std::string path) : path_(std::move(path)) {}

  void load_conf(const std::string& path) { path_ = path; }
  void parse() {
    SS_CHECK_MSG(!path_.empty(), "load_conf(path) first");
    std::set<std::string> stack;
    parse_file(path_, stack);
  }
  void parse_file(const std::string& path) {
    std::set<std::string> stack;
    parse_file(path, stack);
  }
  void parse_string(const std::string& text, const std::string& base_dir = ".") {
    std::set<std::string> stack;
    std::istringstream is(text);
    parse_stream(is, base_dir, stack);
  }

  void clear() { dic_.clear(); }
  bool has(const std::string& key) const { return dic_.count(key) != 0; }
  const Item& get_config(const std::string& key) const {
    auto it = dic_.find(key);
    SS_CHECK_MSG(it != dic_.end(), "no such config key: " << key);
    return it->second;
  }
  std::string get(const std::string& key, const std::string& dflt) const {
    auto it = dic_.find(key);
    return it == dic_.end() ? dflt : it->second.value;
  }
  // first definition wins, like parsing
  bool register_config(const std::string& key, const std::string& value = "") {
    SS_CHECK(!key.empty());
    return dic_.insert({key, Item(value)}).second;
  }
  void set(const std::string& key, const std::string& value) { dic_[key] = Item(value); }
  bool erase(const std::string& key) { return dic_.erase(key) != 0; }
  std::vector<std::pair<std::string, std::string>> items() const {
    std::vector<std::pair<std::string, std::string>> out;
    for (auto& kv : dic_) out.emplace_back(kv.first, kv.second.value);
    return out;
  }
  size_t size() const { return dic_.size(); }
  std::string dump() const {
    std::ostringstream os;
    os << "conf:\n";
    for (auto& kv : dic_) os << kv.first << "\t" << kv.second.value << "\n";
    os << "end conf\n";
    return os.str();
  }
  const std::string& path() const { return path_; }

 private:
  static std::string dirname(const std::string& p) {
    const size_t i = p.find_last_of('/');
    return i == std::string::npos ? "." : (i == 0 ? "/" : p.substr(0, i));
  }
  static bool exists(const std::string& p) {
    std::ifstream f(p);
    return (bool)f;
  }
  void parse_file(const std::string& path, std::set<std::string>& stack) {
    SS_CHECK_MSG(stack.count(path) == 0, "config import cycle at " << path);
    std::ifstream f(path);
    SS_CHECK_MSG((bool)f, "conf can not open: " << path);
    stack.insert(path);
    parse_stream(f, dirname(path), stack);
    stack.erase(path);
  }
  void parse_stream(std::istream& is, const std::string& base, std::set<std::string>& stack) {
    std::string line;
    while (std::getline(is, line)) {
      trim_inplace(line);
      if (line.empty() || startswith(line, "#")) continue;
      if (startswith(line, "import") && line.size() > 6 && (line[6] == ' ' || line[6] == '\t')) {
        std::string p = trim(line.substr(7));
        if (!p.empty() && p[0] != '/' && !exists(p)) p = base + "/" + p;
        parse_file(p, stack);
        continue;
      }
      auto kv = key_value_split(line, ":");
      std::string k = trim(kv.first), v = trim(kv.second);
      SS_CHECK_MSG(!k.empty(), "empty key in config line: " << line);
      dic_.insert({k, Item(v)});
    }
  }

  std::map<std::string, Item> dic_;
  std::string path_;
};

inline ConfigParser& global_config() {
  static ConfigParser cfg;
  return cfg;
}

}  // namespace ss
