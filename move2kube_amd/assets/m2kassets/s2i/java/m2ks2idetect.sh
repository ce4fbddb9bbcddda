#!/bin/sh
# move2kube_amd S2I detector: Java (Maven -> EAP builder, plain sources -> OpenJDK
# builder; Gradle and Ant projects are not handled by S2I).
src="$1"
[ -f "$src/build.gradle" ] && exit 1
[ -f "$src/build.xml" ] && exit 1
if [ -f "$src/pom.xml" ]; then
    printf '{"builder": "%s", "port": 8080}\n' "registry.access.redhat.com/jboss-eap-6/eap64-openshift:latest"
    exit 0
fi
n=$(find "$src"/. -name '*.java' -print 2>/dev/null | head -n 1 | wc -l)
[ "$n" -eq 1 ] || exit 1
printf '{"builder": "%s", "port": 8080}\n' "registry.access.redhat.com/redhat-openjdk-18/openjdk18-openshift:latest"
