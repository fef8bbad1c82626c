// TEST STUB -- not abseil.  absl::Status as the drop-in controller headers and
// tests/cpp/dropin_standing.cpp use it (codes, ok(), message(), Update keeps the first error).
#pragma once
#include <string>
#include <string_view>

namespace absl {
enum class StatusCode : int { kOk = 0, kInvalidArgument = 3, kFailedPrecondition = 9, kInternal = 13 };
class Status {
 public:
  Status() = default;
  Status(StatusCode c, std::string_view m) : code_(c), msg_(m) {}
  bool ok() const { return code_ == StatusCode::kOk; }
  StatusCode code() const { return code_; }
  std::string_view message() const { return msg_; }
  void Update(const Status& s) {
    if (ok() && !s.ok()) *this = s;
  }

 private:
  StatusCode code_ = StatusCode::kOk;
  std::string msg_;
};
inline Status OkStatus() { return Status(); }
inline Status InternalError(std::string_view m) { return Status(StatusCode::kInternal, m); }
inline Status FailedPreconditionError(std::string_view m) { return Status(StatusCode::kFailedPrecondition, m); }
inline Status InvalidArgumentError(std::string_view m) { return Status(StatusCode::kInvalidArgument, m); }
}  // namespace absl
