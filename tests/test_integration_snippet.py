"""INTEGRATION.md §3 (the hand-off table) compiles as written, under -fno-common.

The reference defines its rx counters in tcp_in.c:18-19 and declares them extern in
tcp_in.h:7,11; tcp_in.c stays linked in the patched stack.  So the patch must only refer to
them: an object that also defined them would be a second definition, which links only with
-fcommon (the reference's Makefile era) and fails under gcc >= 10's default -fno-common.

The snippet is extracted from INTEGRATION.md and compiled to an object (-c: no link, so no
stand-in definitions of the reference's functions).  The include it names, "tcp_in.h", is
supplied as the declarations the snippet uses, each with the reference's signature
(file:line below); then nm shows the two counters as undefined references.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Declarations the §3 block relies on (the reference's own prototypes, DPDK types opaque).
DECLS = r"""
#include <stdint.h>
struct rte_mbuf; struct ipv4_hdr; struct tcp_hdr;
struct tcb { uint32_t max_seq_received; };              /* tcp_tcb.h:15-56 (field used) */
extern struct tcb *tcbs[];                             /* tcp_tcb.c:22 */
typedef int (*tcpinstate)(struct tcb *, struct tcp_hdr *, struct ipv4_hdr *, struct rte_mbuf *); /* tcp_states.h:19 */
extern tcpinstate tcpswitch[];                         /* tcp_states.h:32 */
void free_mbuf(struct rte_mbuf *m);                    /* main.h:48 */
int arp_in(struct rte_mbuf *m);                        /* arp.h:60 */
int get_mac(uint32_t ip, unsigned char *mac);          /* arp.c:215 */
int add_mac(uint32_t ip, unsigned char *mac);          /* arp.c:282 */
void send_reset(struct ipv4_hdr *ip, struct tcp_hdr *tcp);   /* tcp_out.c:103 */
void AdjustSendWindow(struct tcb *p, uint32_t ack);    /* tcp_windows.h:70 */
extern int tcpchecksumerror;                           /* tcp_in.h:7 */
extern int tcpnopcb;                                   /* tcp_in.h:11 */
"""


def _snippet():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text.split("## 3. The hand-off table", 1)[1].split("\n## ", 1)[0]
    blocks = re.findall(r"```c\n(.*?)```", sec, re.S)
    code = [b for b in blocks if "rxg_handoff_ops" in b]
    assert len(code) == 1, "INTEGRATION.md §3 must hold one C block with the hand-off table"
    return code[0]


def test_snippet_refers_to_the_reference_counters_only():
    code = _snippet()
    assert '#include "tcp_in.h"' in code
    assert not re.search(r"^\s*int\s+tcp(nopcb|checksumerror)\s*;", code, re.M), \
        "the patch must not define tcp_in.c's counters"


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("nm") is None, reason="gcc/nm missing")
def test_snippet_compiles_fno_common(tmp_path):
    code = _snippet()
    (tmp_path / "tcp_in.h").write_text(DECLS)
    src = tmp_path / "handoff.c"
    # the snippet's callbacks ignore their `u` argument, as the reference has no user data
    src.write_text('#include "rxg.h"\n' + code + "\nconst rxg_handoff_ops *patch_ops(void) { return &g_ops; }\n")
    obj = tmp_path / "handoff.o"
    subprocess.run(["gcc", "-std=gnu11", "-fno-common", "-Wall", "-Werror", "-Wno-unused-parameter",
                    "-I", str(tmp_path), "-I", os.path.join(ROOT, "include"), "-c", str(src), "-o", str(obj)],
                   check=True)
    syms = subprocess.run(["nm", str(obj)], check=True, capture_output=True, text=True).stdout
    kinds = {line.split()[-1]: line.split()[-2] for line in syms.splitlines() if line.split()}
    assert kinds.get("tcpnopcb") == "U" and kinds.get("tcpchecksumerror") == "U", syms
