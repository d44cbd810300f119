// core_test.cc — JSON DOM + patches, YAML, quantities / time, selectors.
#include <cmath>

#include "apiserver/selector.h"
#include "core/json.h"
#include "core/util.h"
#include "core/yaml.h"
#include "tests/harness.h"

using kf::Json;

TEST(json, parse_dump_roundtrip) {
  const std::string text = R"({"a":1,"b":[true,null,"x\né"],"c":{"d":-2.5,"e":"☃"}})";
  Json j = Json::parse(text);
  CHECK_EQ(j["a"].as_int(), 1);
  CHECK(j["b"][1].is_null());
  CHECK_EQ(j["b"][2].as_string(), std::string("x\n\xc3\xa9"));
  CHECK_EQ(j.at_path({"c", "d"}).as_double(), -2.5);
  CHECK(Json::parse(j.dump()) == j);
  Json bad;
  CHECK(!Json::try_parse("{\"a\":", bad));
  CHECK(!Json::try_parse("[1,]", bad));
}

TEST(json, merge_patch_rfc7386_examples) {
  // RFC 7386 appendix A
  CHECK(kf::merge_patch(Json::parse(R"({"a":"b"})"), Json::parse(R"({"a":"c"})")) == Json::parse(R"({"a":"c"})"));
  CHECK(kf::merge_patch(Json::parse(R"({"a":"b"})"), Json::parse(R"({"a":null})")) == Json::parse("{}"));
  CHECK(kf::merge_patch(Json::parse(R"({"a":[{"b":"c"}]})"), Json::parse(R"({"a":[1]})")) == Json::parse(R"({"a":[1]})"));
  CHECK(kf::merge_patch(Json::parse(R"({"e":null})"), Json::parse(R"({"a":1})")) == Json::parse(R"({"e":null,"a":1})"));
  CHECK(kf::merge_patch(Json::parse(R"({})"), Json::parse(R"({"a":{"bb":{"ccc":null}}})")) == Json::parse(R"({"a":{"bb":{}}})"));
  const Json from = Json::parse(R"({"a":1,"b":{"c":2,"d":3},"e":[1,2]})");
  const Json to = Json::parse(R"({"a":1,"b":{"c":5},"e":[3],"f":"n"})");
  CHECK(kf::merge_patch(from, kf::diff_merge_patch(from, to)) == to);
}

TEST(json, json_patch_ops_and_diff) {
  const Json doc = Json::parse(R"({"foo":["bar","baz"],"a/b":{"~c":1}})");
  Json out = kf::apply_json_patch(doc, Json::parse(R"([
    {"op":"add","path":"/foo/1","value":"qux"},
    {"op":"remove","path":"/foo/0"},
    {"op":"replace","path":"/a~1b/~0c","value":2},
    {"op":"copy","from":"/foo","path":"/copied"},
    {"op":"move","from":"/copied","path":"/moved"},
    {"op":"add","path":"/foo/-","value":"end"},
    {"op":"test","path":"/moved/0","value":"qux"}])"));
  CHECK(out == Json::parse(R"({"foo":["qux","baz","end"],"a/b":{"~c":2},"moved":["qux","baz"]})"));
  bool threw = false;
  try {
    kf::apply_json_patch(doc, Json::parse(R"([{"op":"test","path":"/foo/0","value":"nope"}])"));
  } catch (const kf::JsonError&) {
    threw = true;
  }
  CHECK(threw);
  const Json to = Json::parse(R"({"foo":["bar","zap"],"x":{"y":[1,{"z":2}]}})");
  CHECK(kf::apply_json_patch(doc, kf::diff_json_patch(doc, to)) == to);
}

TEST(json, strategic_merge_containers_by_name) {
  const Json pod = Json::parse(R"({"spec":{"containers":[{"name":"a","image":"i1","env":[{"name":"X","value":"1"}]},
                                                         {"name":"b","image":"i2"}],
                                           "tolerations":[{"key":"k1"}]}})");
  const Json patch = Json::parse(R"({"spec":{"containers":[{"name":"a","env":[{"name":"Y","value":"2"}]},
                                                           {"name":"c","image":"i3"}],
                                             "tolerations":[{"key":"k2"}]}})");
  Json out = kf::strategic_merge_patch(pod, patch);
  const auto& cs = out.at_path({"spec", "containers"}).as_array();
  REQUIRE(cs.size() == 3);
  CHECK_EQ(cs[0]["image"].as_string(), std::string("i1"));
  CHECK_EQ(cs[0]["env"].as_array().size(), static_cast<size_t>(2));  // env merges by name
  CHECK_EQ(cs[2]["name"].as_string(), std::string("c"));
  CHECK_EQ(out.at_path({"spec", "tolerations"}).as_array().size(), static_cast<size_t>(1));  // replaced
  Json del = kf::strategic_merge_patch(pod, Json::parse(R"({"spec":{"containers":[{"name":"b","$patch":"delete"}]}})"));
  CHECK_EQ(del.at_path({"spec", "containers"}).as_array().size(), static_cast<size_t>(1));
}

TEST(yaml, documents_block_scalars_roundtrip) {
  std::vector<Json> docs;
  std::string err;
  REQUIRE(kf::parse_yaml_all("a: 1\nb:\n  - x\n  - {k: v}\nc: |\n  line1\n  line2\n---\nkind: Pod\nmetadata:\n  name: 'p-0'\n", docs, &err));
  REQUIRE(docs.size() == 2);
  CHECK_EQ(docs[0]["a"].as_int(), 1);
  CHECK_EQ(docs[0]["b"][1]["k"].as_string(), std::string("v"));
  CHECK_EQ(docs[0]["c"].as_string(), std::string("line1\nline2\n"));
  CHECK_EQ(docs[1].at_path({"metadata", "name"}).as_string(), std::string("p-0"));
  const Json obj = Json::parse(R"({"s":"true","n":3,"l":["a: b","- c"],"m":{"empty":{}},"e":[]})");
  Json back;
  REQUIRE(kf::parse_yaml(kf::dump_yaml(obj), back, &err));
  CHECK(back == obj);
}

TEST(util, quantities_and_time) {
  CHECK_EQ(*kf::parse_quantity("500m"), 0.5);
  CHECK_EQ(*kf::parse_quantity("2Gi"), 2.0 * 1024 * 1024 * 1024);
  CHECK_EQ(*kf::parse_quantity("1e3"), 1000.0);
  CHECK_EQ(*kf::parse_quantity("288Gi") / (1024.0 * 1024 * 1024), 288.0);
  CHECK(!kf::parse_quantity("1 Gi"));
  CHECK(!kf::parse_quantity("abc"));
  CHECK_EQ(kf::rfc3339_from_ms(1700000000123LL, true), std::string("2023-11-14T22:13:20.123Z"));
  CHECK_EQ(*kf::parse_rfc3339_ms("2023-11-14T22:13:20.123Z"), 1700000000123LL);
  CHECK_EQ(*kf::parse_rfc3339_ms("2023-11-14T22:13:20Z"), 1700000000000LL);
  CHECK_EQ(kf::base64_decode(kf::base64_encode(std::string("\x00\xff pem\n", 7))), std::string("\x00\xff pem\n", 7));
  CHECK_EQ(kf::to_upper("cpx"), std::string("CPX"));
}

TEST(selector, label_and_field_selectors) {
  kf::LabelSelector s;
  REQUIRE(kf::LabelSelector::parse("app=nb,tier in (a,b),!legacy,env!=prod", s));
  CHECK(s.matches(Json::parse(R"({"app":"nb","tier":"a","env":"dev"})")));
  CHECK(!s.matches(Json::parse(R"({"app":"nb","tier":"c"})")));
  CHECK(!s.matches(Json::parse(R"({"app":"nb","tier":"a","legacy":"1"})")));
  CHECK(!s.matches(Json::parse(R"({"app":"nb","tier":"b","env":"prod"})")));
  kf::LabelSelector bad;
  CHECK(!kf::LabelSelector::parse("a in (b", bad));
  // PodDefault semantics: a null selector matches nothing; {} matches everything
  CHECK(!kf::LabelSelector::from_json(Json(), true).matches(Json::parse(R"({"x":"y"})")));
  CHECK(kf::LabelSelector::from_json(Json::object(), true).matches(Json::parse(R"({"x":"y"})")));
  const auto e = kf::LabelSelector::from_json(Json::parse(R"({"matchExpressions":[{"key":"gpu","operator":"Exists"}]})"));
  CHECK(e.matches(Json::parse(R"({"gpu":"8"})")) && !e.matches(Json::object()));
  kf::FieldSelector f;
  REQUIRE(kf::FieldSelector::parse("metadata.name=nb-0,status.phase!=Failed", f));
  CHECK(f.matches(Json::parse(R"({"metadata":{"name":"nb-0"},"status":{"phase":"Running"}})")));
  CHECK(!f.matches(Json::parse(R"({"metadata":{"name":"nb-0"},"status":{"phase":"Failed"}})")));
}
