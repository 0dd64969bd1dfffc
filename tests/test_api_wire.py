"""kubelet device-plugin v1beta1 wire compatibility (golden bytes against upstream api.proto).

Field numbers/types of k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto; the bytes
below are hand-encoded from the proto wire format, independent of our descriptor code.
"""
from aliyun_gpushare_device_plugin_amd.api import v1beta1 as api


def test_device_golden_bytes():
    d = api.Device(ID="x", health="Healthy")
    assert d.SerializeToString() == bytes.fromhex("0a0178") + bytes([0x12, 7]) + b"Healthy"
    d.topology.nodes.add(ID=1)
    # field 3 (topology) -> TopologyInfo{field 1 (nodes) -> NUMANode{field 1 int64 = 1}}
    assert d.SerializeToString().endswith(bytes.fromhex("1a04" "0a02" "0801"))


def test_register_request_golden_bytes():
    r = api.RegisterRequest(version="v1beta1", endpoint="aliyungpushare.sock", resource_name="aliyun.com/gpu-mem")
    want = (b"\x0a\x07v1beta1" + b"\x12\x13aliyungpushare.sock" + b"\x1a\x12aliyun.com/gpu-mem")
    assert r.SerializeToString() == want
    r.options.get_preferred_allocation_available = True
    assert r.SerializeToString() == want + bytes.fromhex("2202" "1001")


def test_allocate_request_response_fields():
    req = api.AllocateRequest(container_requests=[api.ContainerAllocateRequest(devices_ids=["a", "b"])])
    assert req.SerializeToString() == bytes.fromhex("0a06" "0a0161" "0a0162")
    resp = api.ContainerAllocateResponse(envs={"K": "V"})
    resp.mounts.add(container_path="/c", host_path="/h", read_only=True)
    resp.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
    resp.annotations["a"] = "b"
    resp.cdi_devices.add(name="amd.com/gpu=0")
    b = resp.SerializeToString()
    # envs map entry (field 1), mounts (2), devices (3), annotations (4), cdi_devices (5)
    assert b[0] == 0x0a and bytes.fromhex("0a014b") in b and bytes.fromhex("120156") in b
    tags = set()
    i = 0
    while i < len(b):
        tag = b[i]
        tags.add(tag >> 3)
        ln = b[i + 1]
        i += 2 + ln
    assert tags == {1, 2, 3, 4, 5}
    assert api.ContainerAllocateResponse.FromString(b) == resp


def test_preferred_allocation_messages():
    r = api.PreferredAllocationRequest(container_requests=[api.ContainerPreferredAllocationRequest(
        available_deviceIDs=["a"], must_include_deviceIDs=["b"], allocation_size=2)])
    assert r.SerializeToString() == bytes.fromhex("0a08" "0a0161" "120162" "1802")
    p = api.ContainerPreferredAllocationResponse(deviceIDs=["z"])
    assert p.SerializeToString() == bytes.fromhex("0a017a")


def test_options_and_empty():
    assert api.Empty().SerializeToString() == b""
    o = api.DevicePluginOptions(pre_start_required=True, get_preferred_allocation_available=True)
    assert o.SerializeToString() == bytes.fromhex("0801" "1001")


def test_method_paths():
    assert api.method_path("DevicePlugin", "Allocate") == "/v1beta1.DevicePlugin/Allocate"
    assert api.method_path("Registration", "Register") == "/v1beta1.Registration/Register"
    names = [m[0] for m in api.SERVICES["DevicePlugin"]]
    assert names == ["GetDevicePluginOptions", "ListAndWatch", "GetPreferredAllocation", "Allocate",
                     "PreStartContainer"]
    assert [m for m in api.SERVICES["DevicePlugin"] if m[3]] == [("ListAndWatch", "Empty",
                                                                 "ListAndWatchResponse", True)]
    svc = api.FILE_DESCRIPTOR.services_by_name["DevicePlugin"]
    assert svc.full_name == "v1beta1.DevicePlugin"


def test_podresources_golden_bytes_and_paths():
    """k8s.io/kubelet/pkg/apis/podresources/v1/api.proto: PodResources{name=1, namespace=2,
    containers=3{name=1, devices=2{resource_name=1, device_ids=2}}}; unknown fields (DRA's
    dynamic_resources) are skipped by the parser."""
    from aliyun_gpushare_device_plugin_amd.api import podresources as pr

    d = pr.ContainerDevices(resource_name="r", device_ids=["a"])
    assert d.SerializeToString() == bytes.fromhex("0a0172" "120161")
    c = pr.ContainerResources(name="c", devices=[d])
    assert c.SerializeToString() == bytes.fromhex("0a0163" "1206") + d.SerializeToString()
    p = pr.PodResources(name="p", namespace="n", containers=[c])
    assert p.SerializeToString() == bytes.fromhex("0a0170" "12016e" "1a0b") + c.SerializeToString()
    # the same container with a DRA dynamic_resources entry (field 5) the plugin does not model
    c_dra = c.SerializeToString() + bytes.fromhex("2a00")
    raw = bytes.fromhex("0a0170" "12016e" "1a0d") + c_dra
    resp = pr.ListPodResourcesResponse.FromString(bytes([0x0a, len(raw)]) + raw)
    assert pr.pod_devices(resp, "r") == [pr.PodDevices("n", "p", (("c", ("a",)),))]
    assert pr.pod_devices(resp, "other") == []
    assert pr.PROTO.method_path("PodResourcesLister", "List") == "/v1.PodResourcesLister/List"
    assert pr.FILE_DESCRIPTOR.services_by_name["PodResourcesLister"].full_name == "v1.PodResourcesLister"
    g = pr.GetPodResourcesRequest(pod_name="p", pod_namespace="n")
    assert g.SerializeToString() == bytes.fromhex("0a0170" "12016e")
