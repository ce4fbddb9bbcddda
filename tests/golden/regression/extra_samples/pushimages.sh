#   Copyright IBM Corporation 2020
#
#   Licensed under the Apache License, Version 2.0 (the "License");
#   you may not use this file except in compliance with the License.
#   You may obtain a copy of the License at
#
#        http://www.apache.org/licenses/LICENSE-2.0
#
#   Unless required by applicable law or agreed to in writing, software
#   distributed under the License is distributed on an "AS IS" BASIS,
#   WITHOUT WARRANTIES OR CONDITIONS OF ANY KIND, either express or implied.
#   See the License for the specific language governing permissions and
#   limitations under the License.

# Invoke as pushimages.sh <registry_url> <registry_namespace>

if [ "$#" -ne 2 ]; then
    REGISTRY_URL=docker.io
    REGISTRY_NAMESPACE=samples
else
    REGISTRY_URL=$1
    REGISTRY_NAMESPACE=$2
fi

# Uncomment the below line if you want to enable login before pushing
# docker login ${REGISTRY_URL}

docker tag samples-compose-api:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/samples-compose-api:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/samples-compose-api:latest
docker tag samples-compose-web:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/samples-compose-web:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/samples-compose-web:latest
docker tag samples-dockerfile:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/samples-dockerfile:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/samples-dockerfile:latest
docker tag sample/api:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/sample/api:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/sample/api:latest
docker tag sample/web:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/sample/web:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/sample/web:latest
docker tag cf-hello:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/cf-hello:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/cf-hello:latest
docker tag compose:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/compose:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/compose:latest
docker tag dockerfile:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/dockerfile:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/dockerfile:latest
docker tag golang:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/golang:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/golang:latest
docker tag java-gradle:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-gradle:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-gradle:latest
docker tag java-maven:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-maven:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/java-maven:latest
docker tag nodejs:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/nodejs:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/nodejs:latest
docker tag php:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/php:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/php:latest
docker tag python:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/python:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/python:latest
docker tag ruby:latest ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/ruby:latest
docker push ${REGISTRY_URL}/${REGISTRY_NAMESPACE}/ruby:latest
