// main.cc — runs the registered native unit tests: [--filter=<suite>] [--list]
#include <cstring>
#include <exception>

#include "tests/harness.h"

int main(int argc, char** argv) {
  std::string filter;
  bool list = false;
  for (int i = 1; i < argc; ++i) {
    if (std::strncmp(argv[i], "--filter=", 9) == 0) filter = argv[i] + 9;
    if (std::strcmp(argv[i], "--list") == 0) list = true;
  }
  int run = 0, failed_cases = 0;
  for (const auto& c : kft::registry()) {
    if (!filter.empty() && c.suite != filter) continue;
    if (list) {
      std::printf("%s.%s\n", c.suite.c_str(), c.name.c_str());
      continue;
    }
    const int before = kft::failures();
    try {
      c.fn();
    } catch (const kft::Abort&) {
    } catch (const std::exception& e) {
      kft::fail(__FILE__, __LINE__, std::string("uncaught exception: ") + e.what());
    }
    ++run;
    const bool ok = kft::failures() == before;
    if (!ok) ++failed_cases;
    std::printf("%s %s.%s\n", ok ? "ok  " : "FAIL", c.suite.c_str(), c.name.c_str());
  }
  if (list) return 0;
  std::printf("%d cases, %d failed\n", run, failed_cases);
  return run == 0 || failed_cases ? 1 : 0;
}
