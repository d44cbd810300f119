// harness.h — the native unit-test harness ("a ctest macro harness"): TEST(suite,
// name) registers a case, CHECK / CHECK_EQ record failures without aborting the case, REQUIRE
// stops it. One binary (kfamd_native_tests) holds every suite; `ctest` runs it once per suite via
// --filter=<suite> so a failure names its suite, and tests/test_native_unit.py runs it under pytest.
#pragma once

#include <cstdio>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

namespace kft {

struct Case {
  std::string suite, name;
  std::function<void()> fn;
};
inline std::vector<Case>& registry() {
  static std::vector<Case> r;
  return r;
}
struct Registrar {
  Registrar(const char* s, const char* n, std::function<void()> f) { registry().push_back({s, n, std::move(f)}); }
};
inline int& failures() {
  static int f = 0;
  return f;
}
struct Abort {};
inline void fail(const char* file, int line, const std::string& what) {
  ++failures();
  std::fprintf(stderr, "  %s:%d: %s\n", file, line, what.c_str());
}
template <typename A, typename B>
std::string show(const A& a, const B& b) {
  std::ostringstream o;
  o << "expected " << b << ", got " << a;
  return o.str();
}

}  // namespace kft

#define KFT_CAT2(a, b) a##b
#define KFT_CAT(a, b) KFT_CAT2(a, b)
#define TEST(suite, name)                                                                              \
  static void KFT_CAT(test_, KFT_CAT(suite, name))();                                                  \
  static kft::Registrar KFT_CAT(reg_, KFT_CAT(suite, name))(#suite, #name, KFT_CAT(test_, KFT_CAT(suite, name))); \
  static void KFT_CAT(test_, KFT_CAT(suite, name))()
#define CHECK(cond) \
  do {              \
    if (!(cond)) kft::fail(__FILE__, __LINE__, "CHECK(" #cond ")"); \
  } while (0)
#define CHECK_EQ(a, b)                                                   \
  do {                                                                   \
    const auto& kft_a = (a);                                             \
    const auto& kft_b = (b);                                             \
    if (!(kft_a == kft_b)) kft::fail(__FILE__, __LINE__, #a " == " #b ": " + kft::show(kft_a, kft_b)); \
  } while (0)
#define REQUIRE(cond)                                                      \
  do {                                                                     \
    if (!(cond)) {                                                         \
      kft::fail(__FILE__, __LINE__, "REQUIRE(" #cond ")");                \
      throw kft::Abort{};                                                  \
    }                                                                      \
  } while (0)
