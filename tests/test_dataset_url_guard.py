"""dataset_url is fetched by the API server: loopback / private / link-local targets (cluster
services, the cloud metadata endpoint) are refused on every hop, redirects included."""
import httpx
import pytest

from finetune_controller_amd.controlplane.tasks import services


@pytest.mark.parametrize("url", ["http://127.0.0.1/x.csv", "http://localhost:8080/x", "http://10.0.0.5/d.jsonl",
                                 "http://169.254.169.254/latest/meta-data/", "http://[::1]/x", "http://192.168.1.2/",
                                 "http://[::ffff:10.1.2.3]/x"])
def test_non_public_targets_are_refused(url):
    with pytest.raises(services.BlockedURL):
        services.guard_url(httpx.Request("GET", url))


def test_public_target_passes_and_redirect_into_the_cluster_is_refused():
    services.guard_url(httpx.Request("GET", "http://93.184.216.34/data.csv"))  # a public literal

    def handler(req):
        if req.url.host == "93.184.216.34":
            return httpx.Response(302, headers={"Location": "http://10.96.0.1/secrets"})
        return httpx.Response(200, content=b"internal")

    with services._http_client(transport=httpx.MockTransport(handler)) as c:
        with pytest.raises(services.BlockedURL):
            c.get("http://93.184.216.34/data.csv")
    # the opt-out for deployments whose datasets live on an internal host
    with services._http_client(allow_private=True, transport=httpx.MockTransport(handler)) as c:
        assert c.get("http://93.184.216.34/data.csv").content == b"internal"


@pytest.mark.parametrize("ip", ["100.64.0.10", "100.100.100.200", "192.0.0.8", "198.18.0.1", "[fd00::1]",
                                "[fe80::1]"])
def test_shared_and_special_ranges_are_refused(ip):
    """100.64.0.0/10 (carrier-grade NAT / some metadata endpoints and CNI pod ranges) and the
    other non-global special ranges are refused, not only RFC 1918."""
    with pytest.raises(services.BlockedURL):
        services.guard_url(httpx.Request("GET", f"http://{ip}/x"))


def test_dns_rebinding_cannot_redirect_the_connection():
    """The name is resolved ONCE per hop and the connection goes to that checked address: a resolver
    that answers public first and metadata second never gets its second answer used, and a resolver that
    answers a private address is refused before any connection."""
    answers = iter([["93.184.216.34"], ["169.254.169.254"]])
    calls = []

    def rebinding(host):
        calls.append(host)
        return next(answers)

    seen = []

    def handler(req):
        seen.append((req.url.host, req.headers["host"], req.extensions.get("sni_hostname")))
        return httpx.Response(200, content=b"ok")

    with services._http_client(transport=httpx.MockTransport(handler), resolve=rebinding) as c:
        assert c.get("http://data.example.org/d.csv").content == b"ok"
    assert calls == ["data.example.org"]  # one resolution, the checked one
    assert seen == [("93.184.216.34", "data.example.org", "data.example.org")]

    with services._http_client(transport=httpx.MockTransport(handler), resolve=lambda h: ["100.64.1.1"]) as c:
        with pytest.raises(services.BlockedURL):
            c.get("http://data.example.org/d.csv")
    assert len(seen) == 1  # refused before the transport connected
