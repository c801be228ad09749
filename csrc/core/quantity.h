// SPDX-License-Identifier: Apache-2.0
// Kubernetes resource.Quantity arithmetic (subset) for PodGroup minResources.
// Parses "2", "500m", "1.5", "4Gi", "10k", "1e3"; sums keep the first
// operand's format; String() follows the canonical forms of apimachinery
// (largest exact suffix; milli fallback for non-integers).
#pragma once

#include <string>

namespace pdo {

class Quantity {
 public:
  enum class Format { DecimalSI, BinarySI, DecimalExponent };
  Quantity() = default;
  static bool parse(const std::string& s, Quantity* out);
  void add(const Quantity& o) { milli_ += o.milli_; }
  std::string str() const;
  long double value() const { return (long double)milli_ / 1000.0L; }
  __int128 milli() const { return milli_; }
  Format format() const { return fmt_; }

 private:
  __int128 milli_ = 0;  // value × 1000 (sub-milli precision is rounded up like Go's)
  Format fmt_ = Format::DecimalSI;
};

}  // namespace pdo
