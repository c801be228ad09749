// SPDX-License-Identifier: Apache-2.0
#include "schema.h"

#include "store.h"

namespace pdo {
namespace schema {

static bool preserve(const Value& s) { return s.get("x-kubernetes-preserve-unknown-fields").as_bool(); }

void prune(Value& v, const Value& s, bool root) {
  if (v.is_object() && (s.get("type").as_string() == "object" || s.has("properties"))) {
    const Value* props = s.find("properties");
    const Value* addl = s.find("additionalProperties");
    if (addl && !addl->is_object()) addl = nullptr;
    json::Object kept;
    for (auto& m : v.obj()) {
      if (root && m.first == "metadata") {
        kept.push_back(std::move(m));
        continue;
      }
      const Value* sub = props ? props->find(m.first) : nullptr;
      if (sub) {
        prune(m.second, *sub, false);
      } else if (addl) {
        prune(m.second, *addl, false);
      } else if (!preserve(s)) {
        continue;  // unknown field: pruned
      }
      kept.push_back(std::move(m));
    }
    v.obj() = std::move(kept);
    return;
  }
  const Value* items = s.find("items");
  if (v.is_array() && items && items->is_object())
    for (auto& e : v.arr()) prune(e, *items, false);
}

static bool type_ok(const Value& v, const Value& s) {
  if (const Value* any = s.find("anyOf")) {
    for (auto& alt : any->arr())
      if (type_ok(v, alt)) return true;
    return false;
  }
  const std::string& t = s.get("type").as_string();
  if (t.empty()) return true;
  if (t == "object") return v.is_object();
  if (t == "array") return v.is_array();
  if (t == "string") return v.is_string();
  if (t == "integer") return v.is_int();
  if (t == "number") return v.is_number();
  if (t == "boolean") return v.is_bool();
  return true;
}

void check(const Value& v, const Value& s, const std::string& path, std::vector<std::string>* errs) {
  if (v.is_null()) return;  // omitempty / explicit null of an optional field
  if (!type_ok(v, s)) {
    const std::string& t = s.get("type").as_string();
    errs->push_back((path.empty() ? "<root>" : path) + ": Invalid value: must be of type " +
                    (t.empty() ? "int-or-string" : t));
    return;
  }
  const std::string pre = path.empty() ? "" : path + ".";
  if (v.is_object()) {
    for (auto& r : s.get("required").arr()) {
      const Value* f = v.find(r.as_string());
      if (!f || f->is_null()) errs->push_back(pre + r.as_string() + ": Required value");
    }
    const Value* props = s.find("properties");
    const Value* addl = s.find("additionalProperties");
    for (auto& m : v.obj()) {
      const Value* sub = props ? props->find(m.first) : nullptr;
      if (sub) check(m.second, *sub, pre + m.first, errs);
      else if (addl && addl->is_object()) check(m.second, *addl, pre + m.first, errs);
    }
  } else if (v.is_array()) {
    const Value* items = s.find("items");
    if (items && items->is_object()) {
      size_t i = 0;
      for (auto& e : v.arr()) check(e, *items, path + "[" + std::to_string(i++) + "]", errs);
    }
  }
}

static const char kSchemaJson[] =
#include "crd_schema.inc"
    ;

const Value& paddlejob_schema() {
  static const Value s = Value::parse(kSchemaJson);
  return s;
}

void admit_paddlejob(Value& obj) {
  const Value& s = paddlejob_schema();
  prune(obj, s, true);
  std::vector<std::string> errs;
  check(obj, s, "", &errs);
  if (!errs.empty()) {
    std::string msg = "PaddleJob.batch.paddlepaddle.org \"" + obj.at_path("metadata.name").str() + "\" is invalid: ";
    for (size_t i = 0; i < errs.size(); ++i) msg += (i ? ", " : "") + errs[i];
    throw store::ApiError(store::ApiError::Invalid, msg);
  }
}

}  // namespace schema
}  // namespace pdo
