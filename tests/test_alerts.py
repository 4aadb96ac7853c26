"""The alert rules (``gtk config alerts`` -> deploy/prometheus-rules.yaml) use only metrics, labels and
label values the device plugin and the extender actually export: checked against the expositions of a
running cluster simulation (plugin, extender with its informer), so a renamed metric cannot silently
disable an alert."""
import re
from pathlib import Path

import yaml

from gpu_topology_on_k8s_amd.config import prometheus_rules
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx

REPO = Path(__file__).resolve().parent.parent
SCRAPE_LABELS = {"pod", "instance", "job", "namespace", "node"}  # added by Prometheus, not by the exporters


def _expositions():
    with SimCluster({"n": fx.f7_mi355x()}, informer=True) as c:
        c.submit("p", 2)
        c.schedule_pending()
        return c.nodes["n"].plugin.metrics.exposition().decode() + c.extender.metrics.exposition().decode()


def _samples(text):
    """metric sample name -> label names seen on it."""
    out = {}
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        m = re.match(r"([a-zA-Z_:][a-zA-Z0-9_:]*)(\{([^}]*)\})?", line)
        out.setdefault(m.group(1), set()).update(re.findall(r'([a-zA-Z_][a-zA-Z0-9_]*)="', m.group(3) or ""))
    return out


def test_every_alert_uses_exported_metrics_and_labels():
    samples = _samples(_expositions())
    rules = [r for g in prometheus_rules()["spec"]["groups"] for r in g["rules"]]
    assert len(rules) >= 10 and len({r["alert"] for r in rules}) == len(rules)
    for r in rules:
        expr = r["expr"]
        assert expr.count("(") == expr.count(")") and expr.count("[") == expr.count("]"), r["alert"]
        names = set(re.findall(r"\b(gtk_[a-z_]+)", expr))
        assert names, r["alert"]
        for name in names:
            assert name in samples, (r["alert"], name)
            used = set(re.findall(r"\b([a-z_]+)\s*(?:=~|!=|=)\s*\\?\"", expr)) | \
                {x.strip() for grp in re.findall(r"(?:by|on)\s*\(([^)]*)\)", expr) for x in grp.split(",")}
            assert used - SCRAPE_LABELS <= set().union(*(samples[n] for n in names)) | {"le"}, (r["alert"], used)
        assert r["labels"]["severity"] in ("critical", "warning", "info") and r["annotations"]["description"]


def test_the_allocate_outcomes_an_alert_matches_exist():
    src = (REPO / "gpu_topology_on_k8s_amd" / "deviceplugin" / "plugin.py").read_text()
    expr = next(r["expr"] for g in prometheus_rules()["spec"]["groups"] for r in g["rules"] if r["alert"] == "GPUTopologyAllocateRefused")
    for outcome in re.search(r'outcome=~\\?"([^"\\]+)', expr).group(1).split("|"):
        assert f'"{outcome}")' in src, outcome  # passed to _refuse(...) as its outcome


def test_the_committed_rules_are_the_generated_ones():
    assert yaml.safe_load((REPO / "deploy" / "prometheus-rules.yaml").read_text()) == prometheus_rules()
