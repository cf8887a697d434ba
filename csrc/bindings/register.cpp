// Aggregates the per-family op registrations into the extension module.
#include "ops_decl.h"

namespace sdx_bind {
void register_supcon(pybind11::module& m);
void register_conv_bn(pybind11::module& m);
void register_data(pybind11::module& m);
void register_optim(pybind11::module& m);
void register_pool(pybind11::module& m);
void register_wprep(pybind11::module& m);
void register_xgmi(pybind11::module& m);
void register_comm(pybind11::module& m);
void register_head(pybind11::module& m);
void register_probe(pybind11::module& m);

void register_ops(pybind11::module& m) {
  register_supcon(m);
  register_conv_bn(m);
  register_data(m);
  register_optim(m);
  register_pool(m);
  register_wprep(m);
  register_xgmi(m);
  register_comm(m);
  register_head(m);
  register_probe(m);
}
}  // namespace sdx_bind
