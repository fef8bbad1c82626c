// TEST STUB -- not abseil.  ABSL_CHECK(cond) << msg: abort with the message when cond is false.
#pragma once
#include <cstdlib>
#include <iostream>

namespace absl_stub {
struct CheckFail {
  bool fail;
  ~CheckFail() {
    if (fail) {
      std::cerr << std::endl;
      std::abort();
    }
  }
  template <class T>
  CheckFail& operator<<(const T& v) {
    if (fail) std::cerr << v;
    return *this;
  }
};
}  // namespace absl_stub
#define ABSL_CHECK(cond) absl_stub::CheckFail{!(cond)} << "Check failed: " #cond " "
