/* compatibility path: reference layout hash_table/inc/hash_table.h */
#include "../../hash_table.h"
