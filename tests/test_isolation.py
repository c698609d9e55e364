"""The product never routes through the oracle (CPU only)."""
import ast
import os

PKG = os.path.join(os.path.dirname(os.path.dirname(__file__)), "gnss_sim_receiver_amd")


def test_product_does_not_import_oracle():
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(".py"):
                tree = ast.parse(open(os.path.join(root, f)).read())
                for node in ast.walk(tree):
                    if isinstance(node, ast.Import):
                        assert not any(a.name.split(".")[0] == "oracle" for a in node.names), f
                    if isinstance(node, ast.ImportFrom):
                        assert (node.module or "").split(".")[0] != "oracle", f
            if f.endswith((".hip", ".cpp", ".h")):
                src = open(os.path.join(root, f)).read()
                assert "orc_" not in src and "liboracle" not in src, f
