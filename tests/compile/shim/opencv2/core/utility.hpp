// forwarding header of the compile-test shim (tests/test_compile_boundary.py)
#include "../../lorb_cv_shim.hpp"
