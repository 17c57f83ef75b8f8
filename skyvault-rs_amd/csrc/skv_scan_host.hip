// placeholder
#include "skv_host.hpp"
