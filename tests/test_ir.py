"""IR merge/add rules (cases mirror ``internal/types/ir_test.go``)."""

from move2kube_amd.models import collection
from move2kube_amd.models import ir as irtypes
from move2kube_amd.models import plan as plantypes

DF = plantypes.NEW_DOCKERFILE


def C(name="name1", new=True, images=None, files=None, uid=None):
    c = irtypes.new_container(DF, name, new)
    if images is not None:
        c.image_names = list(images)
    if files:
        c.new_files.update(files)
    if uid is not None:
        c.user_id = uid
    return c


def state(c):
    return (c.container_build_type, c.image_names, c.new, c.new_files, c.exposed_ports, c.user_id, c.accessed_dirs)


def test_add_volume_dedups_by_name():
    s = irtypes.Service()
    s.add_volume({"name": "name1"})
    s.add_volume({"name": "name1"})
    assert s.volumes == [{"name": "name1"}]


def test_new_container():
    c = irtypes.new_container(DF, "name1", True)
    assert c.image_names == ["name1"] and c.new is True and c.new_files == {}


def test_new_container_from_image_info():
    info = collection.ImageInfo()
    info.tags = ["tag1"]
    c = irtypes.new_container_from_image_info(info)
    assert c.image_names == ["tag1"] and c.exposed_ports == info.ports and c.user_id == info.user_id
    c = irtypes.new_container_from_image_info(collection.ImageInfo())
    assert c.image_names == []


def test_merge_unrelated_containers():
    c1, c2 = C(), C("name2")
    assert not c1.merge(c2) and state(c1) == state(C())
    c1 = C(images=["imgname1", "imgname2", "imgname3"])
    assert not c1.merge(C("name2", images=["imgname4", "imgname5", "imgname6"]))
    assert c1.image_names == ["imgname1", "imgname2", "imgname3"]


def test_merge_shared_image_names():
    c1 = C(images=["imgname1", "imgname2", "imgname3"])
    assert c1.merge(C("name2", new=False, images=["imgname3", "imgname4", "imgname5"]))
    assert c1.image_names == ["imgname1", "imgname2", "imgname3", "imgname4", "imgname5"]


def test_merge_new_containers_files_and_users():
    c1 = C(images=["imgname1", "imgname2", "imgname3"], files={"path1": "contents1"}, uid=1)
    assert c1.merge(C("name2", images=["imgname3", "imgname4", "imgname5"], files={"path1": "contents2", "path2": "x"}, uid=2))
    assert c1.new_files == {"path1": "contents1", "path2": "x"} and c1.user_id == 1


def test_merge_new_into_old_takes_files_and_user():
    c1 = C(new=False, images=["imgname1", "imgname2", "imgname3"], files={"path1": "contents1"}, uid=1)
    assert c1.merge(C("name2", images=["imgname3", "imgname4", "imgname5"], files={"path2": "contents2"}, uid=2))
    assert c1.new is False and c1.user_id == 2 and c1.new_files == {"path2": "contents2"}


def test_add_file_port_image_dirs():
    c = C()
    c.add_file("p", "a")
    c.add_file("p", "b")
    assert c.new_files == {"p": "a"}
    c.add_exposed_port(8080)
    c.add_exposed_port(8080)
    assert c.exposed_ports == [8080]
    c.add_image_name("x")
    c.add_image_name("x")
    assert c.image_names == ["name1", "x"]
    c.add_accessed_dirs("/d")
    c.add_accessed_dirs("/d")
    assert c.accessed_dirs == ["/d"]


def test_new_ir():
    ir = irtypes.new_ir(plantypes.new_plan())
    assert ir.containers == [] and ir.services == {} and ir.storages == [] and ir.values.global_variables == {}


def test_ir_merge_names():
    a, b = irtypes.new_ir(plantypes.new_plan()), irtypes.new_ir(plantypes.new_plan())
    a.name, b.name = "name1", "name2"
    a.merge(b)
    assert a.name == "name1"
    a, b = irtypes.new_ir(plantypes.new_plan()), irtypes.new_ir(plantypes.new_plan())
    a.name, b.name = "", "name1"
    a.merge(b)
    assert a.name == "name1"


def test_ir_merge_filled():
    ir1, ir2 = irtypes.new_ir(plantypes.new_plan()), irtypes.new_ir(plantypes.new_plan())
    s1, s2 = irtypes.Service("svcname1"), irtypes.Service("svcname1")
    s1.replicas, s2.replicas = 2, 4
    ir1.services["svcname1"] = s1
    ir2.services["svcname1"] = s2
    c1 = C("contname1", images=["imgname1", "imgname2", "imgname3"])
    ir2.containers.append(c1)
    ir2.storages.append(irtypes.Storage(name="storage1"))
    ir1.merge(ir2)
    assert ir1.services["svcname1"].replicas == 4
    assert [state(c) for c in ir1.containers] == [state(c1)]
    assert [s.name for s in ir1.storages] == ["storage1"]


def test_storage_merge():
    s1, s2 = irtypes.Storage(), irtypes.Storage()
    assert s1.merge(s2)
    s1, s2 = irtypes.Storage(name="name1"), irtypes.Storage(name="name2")
    assert not s1.merge(s2) and s1.name == "name1"
    s1, s2 = irtypes.Storage(content={"key1": b"val1"}), irtypes.Storage(content={"key2": b"val2"})
    assert s1.merge(s2) and s1.content == {"key2": b"val2"}


def test_add_container_and_storage_dedup():
    ir = irtypes.new_ir(plantypes.new_plan())
    ir.add_container(C())
    ir.add_container(C())
    assert len(ir.containers) == 1
    ir.add_storage(irtypes.Storage())
    ir.add_storage(irtypes.Storage())
    assert len(ir.storages) == 1


def test_get_container_by_name_and_url():
    ir = irtypes.new_ir(plantypes.new_plan())
    assert ir.get_container("imgname1")[1] is False
    ir.containers.append(C("contname1"))
    assert ir.get_container("imgname1")[1] is False
    ir.containers[0].image_names.append("imgname1")
    assert ir.get_container("imgname1")[1] is True
    ir.kubernetes.registry_url = "registry1.com"
    assert ir.get_container("registry1.com/namespace/imgname1")[1] is True
