/*
 * topo_parser.h -- drop-in stand-in for the reference's
 * repository/include/topo_parser.h, so that host.c:4's include resolves.
 *
 * The reference declares the controller's YAML topology readers
 * (parse_config, get_switch_info: topo_parser.h:23-24, over yaml-cpp).  There
 * is no controller or switch topology here: the group rendezvous in
 * inccl_group_create replaces both, so nothing is declared.  A caller of those
 * two functions is a switch or controller program, which is out of scope.
 */
#ifndef INCCL_AMD_TOPO_PARSER_H
#define INCCL_AMD_TOPO_PARSER_H

#include "util.h"

#endif /* INCCL_AMD_TOPO_PARSER_H */
