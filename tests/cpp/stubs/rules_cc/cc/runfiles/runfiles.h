// TEST STUB -- not Bazel's runfiles library.  rules_cc::cc::runfiles::Runfiles as the reference's
// examples use it (Create(argv0, BAZEL_CURRENT_REPOSITORY, &error), Rlocation(path)), for
// tests/test_examples_compile.py; defined in tests/cpp/stubs/mujoco_stub.cpp.
#pragma once
#include <string>

namespace rules_cc::cc::runfiles {
class Runfiles {
 public:
  static Runfiles* Create(const std::string& argv0, const std::string& source_repository,
                          std::string* error = nullptr);
  std::string Rlocation(const std::string& path) const;
};
}  // namespace rules_cc::cc::runfiles
