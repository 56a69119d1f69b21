// ORACLE -- TEST INFRASTRUCTURE ONLY. Local BA restatement (filled in later).
#include "ref_lba.h"
