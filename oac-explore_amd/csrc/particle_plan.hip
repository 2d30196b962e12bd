// placeholder -- P-OAC K-head critic plan (filled in below)
#include "oac_common.h"
